#!/bin/bash
# A/B the config-3 bench over env variants on one box (interleaved: a, b, ..., a, b, ...):
#   VARIANTS="name:ENV=VAL,ENV2=VAL2 name2:" ROUNDS=2 BENCH_ARGS="--steps 20" bash tools/gpu_bench_ab.sh
# Each run: python bench.py --no-cpu-baseline $BENCH_ARGS under its own time limit; the JSON lines
# go to gpurun_out/bench_ab/<name>_<round>.json. Stops at the first crash or timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/bench_ab
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-1}); do
  for v in ${VARIANTS:-default:}; do
    name=${v%%:*}; envs=${v#*:}
    (
        IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; unset IFS
        timeout -k 10 ${AB_TIMEOUT:-300} python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} \
            > $O/${name}_$r.json 2> $O/${name}_$r.err
    )
    rc=$?
    echo "== $name round $r rc=$rc: $(grep -o '"value": [0-9.]*' $O/${name}_$r.json | head -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0

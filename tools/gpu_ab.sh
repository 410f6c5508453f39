#!/bin/bash
# A/B one pytest selection over library / env variants on one box:
#   VARIANTS="name:ENV=VAL,ENV2=VAL2 name2:..." bash tools/gpu_ab.sh <pytest args...>
# ENCX_LIB=<file> in a variant picks another build of the library (encx/_lib.py).
# Stops at the first crash or timeout (exit > 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-default:}; do
    name=${v%%:*}; envs=${v#*:}
    (
        IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; unset IFS
        timeout -k 10 ${AB_TIMEOUT:-400} python -u -m pytest "$@" -q -rA -s --timeout 300 --timeout-method thread \
            > gpurun_out/ab_$name.log 2>&1
    )
    rc=$?
    echo "== $name rc=$rc: $(tail -1 gpurun_out/ab_$name.log)"
    [ $rc -gt 1 ] && exit $rc
done
exit 0

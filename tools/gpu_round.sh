#!/bin/bash
# One GPU-box session: parity tests, smoke, bench (+ optional rocprof). Stops at the first
# crash / timeout (exit 124, 134, 137, 139 or a negative signal), continues past plain test
# failures (pytest exit 1) so the log shows every result.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; esac; [ "$1" -ge 128 ] && return 0; return 1; }
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name: $*" | tee -a $OUT/summary.log
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a $OUT/summary.log
    tail -n 40 "$OUT/$name.log"
    if fatal $rc; then echo "FATAL in $name, stopping" | tee -a $OUT/summary.log; exit $rc; fi
    return 0
}
STEPS="${STEPS:-tests smoke bench}"
for s in $STEPS; do
  case $s in
    tests) run tests 1500 python -m pytest tests -m gpu -q -rf --timeout 600 ${PYTEST_ARGS:-} ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ${BENCH_ARGS:-} ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} ;;
  esac
done

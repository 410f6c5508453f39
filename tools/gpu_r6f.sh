#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
export ENCX_LIB=${ENCX_LIB:-encodec-pytorch_amd/stage/r6f.so}
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
ENCX_CONV2=1 step tests_v2 900 python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread
VARIANTS="base: v2:ENCX_CONV2=1" ROUNDS=2 BENCH_ARGS="--steps 20 --no-roofline" step benchab 600 bash tools/gpu_bench_ab.sh
ENCX_CONV2=1 step bench_gen 300 python -u bench.py --config gen --no-cpu-baseline --no-roofline

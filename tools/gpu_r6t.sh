#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
ENCX_MEL_FUSED=0 step m0 300 python -u -m pytest tests/test_gpu_fullsize.py -q -rf -s -k "config3_b32_step" --timeout 250 --timeout-method thread
ENCX_BLAS=0 step b0 300 python -u -m pytest tests/test_gpu_fullsize.py -q -rf -s -k "config3_b32_step" --timeout 250 --timeout-method thread

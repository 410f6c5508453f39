#!/bin/bash
# round-6 session B: conv v2 correctness + per-layer sweep; the audit failures with details
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
ENCX_CONV2=1 step v2tests 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -k "conv_fixture or conv_model_shapes or seanet_layers" -q -rf --timeout 300 --timeout-method thread
SWEEP_STEPS=3 step sweep 500 python -u tools/conv_sweep.py - CONV2=1 CONV2=1,CONV2_RED=32 CONV2=1,CONV2_RED=96 CONV2=1,CONV2_TILE=1 CONV2=1,CONV2_TILE=4 CONV2=1,CONV2_KS=1
step audit 600 python -u -m pytest tests/test_gpu_disc.py tests/test_gpu_48k.py tests/test_gpu_fullsize.py -k "gan_fixture or 48k_fixture or step_vs_oracle" -q -rf --timeout 500 --timeout-method thread

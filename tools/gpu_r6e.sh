#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
export ENCX_LIB=${ENCX_LIB:-encodec-pytorch_amd/stage/r6e.so}
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
ENCX_CONV2=1 step v2tests 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py -k "conv_fixture or conv_model_shapes or seanet_layers" -q -rf --timeout 300 --timeout-method thread
SWEEP_STEPS=3 step sweep 500 python -u tools/conv_sweep.py - CONV2=1 CONV2=1,CONV2_TILE=3 CONV2=1,CONV2_WGS=512 CONV2=1,CONV2_WGS=2048
step flipdiag 300 python -u tools/diag/flip_audit_diag.py
step b32step 600 python -u -m pytest tests/test_gpu_fullsize.py -k "step_vs_oracle" -q -rf --timeout 500 --timeout-method thread

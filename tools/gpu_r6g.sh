#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
export ENCX_LIB=${ENCX_LIB:-encodec-pytorch_amd/stage/r6g.so}
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
step mel 300 python -u -m pytest tests/test_gpu_kernels.py -k "mel or losses" -q -rf --timeout 200 --timeout-method thread
ENCX_CONV2=1 step l48v2 300 python -u -m pytest tests/test_gpu_fullsize.py -k "48k" -q -rf -s --timeout 200 --timeout-method thread
step l48 300 python -u -m pytest tests/test_gpu_fullsize.py -k "48k" -q -rf -s --timeout 200 --timeout-method thread
step audit 600 python -u -m pytest tests/test_gpu_disc.py tests/test_gpu_48k.py tests/test_gpu_model.py -k "gan_fixture or 48k_fixture or b32_step_and_input or 48k_stereo" -q -rf --timeout 500 --timeout-method thread
VARIANTS="v2:ENCX_CONV2=1,ENCX_MEL_FUSED=0 v2mel:ENCX_CONV2=1" ROUNDS=2 BENCH_ARGS="--steps 20 --no-roofline" step benchab 600 bash tools/gpu_bench_ab.sh

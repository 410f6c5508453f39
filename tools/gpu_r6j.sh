#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
export ENCX_LIB=${ENCX_LIB:-encodec-pytorch_amd/stage/r6j.so}
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
for m in 1 2 4; do
ENCX_CONV2=$m step f48_$m 300 python -u -m pytest tests/test_gpu_48k.py -k "forward_48k" -q -rf -s --timeout 200 --timeout-method thread
done
step sweep 400 python tools/conv_sweep.py - CONV2=7 CONV2=7,CONV2_LOWT=1

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
export ENCX_LIB=${ENCX_LIB:-encodec-pytorch_amd/stage/r6j.so}
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
ENCX_CONV2=7 step t48 400 python -u -m pytest tests/test_gpu_48k.py -q -rf -s --timeout 300 --timeout-method thread
ENCX_CONV2=7 step tall 900 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread --deselect tests/test_gpu_48k.py

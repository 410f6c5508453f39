#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
export ENCX_LIB=${ENCX_LIB:-encodec-pytorch_amd/stage/r6g.so}
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
ENCX_CONV2=1 step l48v2 300 python -u -m pytest tests/test_gpu_fullsize.py -k "48k and 4800" -q -rf -s --timeout 200 --timeout-method thread
ENCX_CONV2=1 step f48v2 300 python -u -m pytest tests/test_gpu_48k.py -k "forward_48k" -q -rf -s --timeout 200 --timeout-method thread
export ENCX_CONV2=1
step layers 300 python tools/layer_table.py --config gan

#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
step b1 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -q -rf -s -k "config3_b32_step or resblock or b32" --timeout 250 --timeout-method thread
step layers 300 python tools/layer_table.py --config gen

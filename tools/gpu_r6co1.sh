#!/bin/bash
# Round 6 (late): one-channel kernels -- parity tests, then per-layer tables with and without CO1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/co1
O=gpurun_out/co1
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -2 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
step t 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_disc.py -q -rf --timeout 300 --timeout-method thread -k "conv or seanet or disc or co1 or post or 48k"
step lay1 300 python tools/layer_table.py --config gan
ENCX_CO1=0 step lay0 300 python tools/layer_table.py --config gan
grep -E "32x1|1x32" $O/lay1.log $O/lay0.log

#!/bin/bash
# Round 6 (late): loss-reduction partial blocks -- disc/loss tests, feat rows of the layer table, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lp
O=gpurun_out/lp
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -2 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
step t 400 python -u -m pytest tests/test_gpu_disc.py tests/test_gpu_fullsize.py tests/test_gpu_model.py tests/test_gpu_48k.py -q -rf --timeout 300 --timeout-method thread
step lay 300 python tools/layer_table.py --config gan
step bench 300 python bench.py --no-cpu-baseline

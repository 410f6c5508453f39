#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
ENCX_BLAS=15 step t15 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_kernels.py tests/test_gpu_48k.py -q -rf -s -k "b32 or conv or 48k or mel or losses or lstm" --timeout 300 --timeout-method thread
for b in 3 7 11 15; do ENCX_BLAS=$b step lay$b 300 python tools/layer_table.py --config gen; done
for b in 3 15 3 15; do ENCX_BLAS=$b step bg$b 300 python bench.py --config gen --steps 20 --no-cpu-baseline; grep -o '"value": [0-9.]*' $O/bg$b.log; done

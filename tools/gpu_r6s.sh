#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
step t1 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -q -rf -s -k "b32 or conv or lstm" --timeout 300 --timeout-method thread
step layers 300 python tools/layer_table.py --config gen
step bench_gen 300 python bench.py --config gen --steps 20 --no-cpu-baseline
ENCX_BLAS=0 step bench_gen0 300 python bench.py --config gen --steps 20 --no-cpu-baseline

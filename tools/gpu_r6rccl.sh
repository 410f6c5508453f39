#!/bin/bash
# Round 6 (late): the N > 1 step over a one-rank RCCL group (test + bench line), HEAD bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rccl
O=gpurun_out/rccl
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -2 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
step t 300 python -u -m pytest tests/test_gpu_rccl.py -q -rf -s --timeout 280 --timeout-method thread
ENCX_DIST_FORCE=1 step bench_rccl1 300 python bench.py --no-cpu-baseline
step bench_eager 300 python bench.py --no-cpu-baseline --no-graphs

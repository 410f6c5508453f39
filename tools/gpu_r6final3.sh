#!/bin/bash
# Round-6 end-of-session evidence at HEAD, part 1: GPU tests, smoke, the three bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final3
O=gpurun_out/final3
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -2 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
step tests 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_gan 400 python bench.py
step bench_gen 300 python bench.py --config gen
step bench_48k 400 python bench.py --config 48k

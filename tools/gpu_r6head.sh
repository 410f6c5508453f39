#!/bin/bash
# HEAD check: GPU tests, smoke, config-3 and config-2 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/head
O=gpurun_out/head
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -2 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
step new 300 python -u -m pytest tests/test_gpu_kernels.py -q -rf --timeout 120 --timeout-method thread -k "dilated or many_losses or lstm_vs_oracle or balancer"
step tests 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_gan 400 python bench.py
step bench_gen 300 python bench.py --config gen --no-cpu-baseline

#!/bin/bash
# Round-6 end-of-session evidence at HEAD, part 2: layer tables + rocprofv3 kernel stats (gan, gen),
# three PMC passes of the config-3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -2 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
CONFIG=gan step lay_gan 700 bash tools/gpu_layers.sh
CONFIG=gen step lay_gen 500 bash tools/gpu_layers.sh
BENCH_ARGS="--steps 3 --warmup 1" step pmc 900 bash tools/gpu_pmc.sh

#!/bin/bash
# Round-6 evidence session: layer tables + rocprofv3 kernel-trace stats (gan, gen), three PMC passes
# of the config-3 bench (counters in their own runs), and the two-rank one-GPU rehearsal with and
# without HIP graphs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -2 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
CONFIG=gan step lay_gan 700 bash tools/gpu_layers.sh
CONFIG=gen step lay_gen 500 bash tools/gpu_layers.sh
BENCH_ARGS="--steps 3 --warmup 1" step pmc 900 bash tools/gpu_pmc.sh
export HSA_ENABLE_IPC_MODE_LEGACY=0
ENCX_BENCH_REHEARSE=1 ENCX_DP_GRAPHS=0 step reh_eager 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3
ENCX_BENCH_REHEARSE=1 ENCX_DP_GRAPHS=1 step reh_graphs 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 10 --warmup 3

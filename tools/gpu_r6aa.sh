#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
step t 400 python -u -m pytest tests -m gpu -q -rf -s -k "lstm or config3_b32" --timeout 300 --timeout-method thread
step lay 300 python tools/layer_table.py --config gen
step bg 300 python bench.py --config gen --steps 20 --no-cpu-baseline
export HSA_ENABLE_IPC_MODE_LEGACY=0
ENCX_BENCH_REHEARSE=1 step reh_eager 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3

#!/bin/bash
# Per-layer event table + rocprofv3 kernel-trace summary of one config (CONFIG=gen|gan|48k).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${CONFIG:-gan}
timeout -k 10 300 python tools/layer_table.py --config $C > gpurun_out/layers_$C.md 2> gpurun_out/layers_$C.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$C -o run --output-format csv -- \
    python3 bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$C.log 2>&1 || exit $?
N=1; [ "$C" != gen ] && N=2
python tools/prof_summary.py gpurun_out/prof_$C 60 --adams-per-step $N > gpurun_out/step_kernels_$C.md

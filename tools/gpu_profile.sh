#!/bin/bash
# Evidence pass for one config (CONFIG=gen|gan): rocprofv3 kernel-trace summary of a bench run,
# then FETCH_SIZE and WRITE_SIZE PMC passes (one counter block per run, kernel-trace only, no
# sys/runtime trace), each under its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
C=${CONFIG:-gen}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$C -o run --output-format csv -- \
    python3 bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$C.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF_$C -o run --output-format csv -- \
    python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-graphs > gpurun_out/pmcF_$C.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW_$C -o run --output-format csv -- \
    python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-graphs > gpurun_out/pmcW_$C.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_$C.log

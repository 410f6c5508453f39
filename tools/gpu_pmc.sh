#!/bin/bash
# PMC passes over a short bench run (counters in their own runs, kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-roofline ${BENCH_ARGS:-}"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d gpurun_out/pmc1 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc1.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc2 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc2.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc3 -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc3.log 2>&1

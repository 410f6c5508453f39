#!/bin/bash
# PMC pass over the conv2d microbenchmark (tools/mb/c2_mb) for one layer filter: wave-state,
# MFMA-busy and LDS counters per kernel variant (counters in their own run, kernel-trace only).
# usage: tools/gpu_pmc_mb.sh "d0 L2"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
F=${1:-d0 L2}
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmcmb1 -o run --output-format csv -- tools/mb/c2_mb "$F" > gpurun_out/pmcmb1.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/pmcmb2 -o run --output-format csv -- tools/mb/c2_mb "$F" > gpurun_out/pmcmb2.log 2>&1

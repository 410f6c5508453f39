# round-4 profile: per-layer tables (fused residual block on / off), rocprofv3 kernel trace, PMC
O=gpurun_out/r4_07
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/layer_table.py --config gan > $O/layers_gan.md 2> $O/layers_gan.err || exit $?
ENCX_RESBLOCK=0 timeout -k 10 300 python tools/layer_table.py --config gan > $O/layers_gan_norb.md 2> $O/layers_gan_norb.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_gan -o run --output-format csv -- \
    python3 bench.py --config gan --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_gan.log 2>&1 || exit $?
python tools/prof_summary.py $O/prof_gan 70 --adams-per-step 2 > $O/step_kernels_gan.md
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-roofline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $O/pmc1 -o run --output-format csv -- python3 bench.py $ARGS > $O/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc2 -o run --output-format csv -- python3 bench.py $ARGS > $O/pmc2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $O/pmc3 -o run --output-format csv -- python3 bench.py $ARGS > $O/pmc3.log 2>&1 || exit $?

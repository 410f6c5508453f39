# round-4: fused residual block with register prefetch (buffer loads): parity, per-kernel times, A/B
O=gpurun_out/r4_09
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "resblock" -x -v --timeout 120 --timeout-method thread > $O/rb_tests.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rb -o run --output-format csv -- python3 tools/diag/rb_bench.py 10 > $O/prof_rb.log 2>&1 || exit $?
ENCX_RESBLOCK=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_norb -o run --output-format csv -- python3 tools/diag/rb_bench.py 10 > $O/prof_norb.log 2>&1 || exit $?
VARIANTS="rb: norb:ENCX_RESBLOCK=0" ROUNDS=2 BENCH_ARGS="--steps 20" bash tools/gpu_bench_ab.sh > $O/ab.txt 2>&1

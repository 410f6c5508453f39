# round-4: reworked fused residual block (fwd / dgrad / wgrad kernels): parity, then A/B vs unfused
O=gpurun_out/r4_08
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "resblock" -x -v --timeout 120 --timeout-method thread > $O/rb_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/layer_table.py --config gan > $O/layers_gan.md 2> $O/layers_gan.err || exit $?
VARIANTS="rb: norb:ENCX_RESBLOCK=0" ROUNDS=2 BENCH_ARGS="--steps 20" bash tools/gpu_bench_ab.sh > $O/ab.txt 2>&1

mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_48k.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -5 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/layer_table.py > gpurun_out/layers_gen.md 2>gpurun_out/layers.err || exit $?
head -40 gpurun_out/layers_gen.md; tail -2 gpurun_out/layers_gen.md
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1

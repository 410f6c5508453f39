# round-4: FFT spectrogram tests, then bench evidence: fused resblock A/B, FFT A/B, config 2 /
# config 5 lines, eager N=1, 2-rank rehearsal
O=gpurun_out/r4_06
mkdir -p $O
rc=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_disc.py -x -v --timeout 300 --timeout-method thread -s -k "spectrogram or mel or losses or disc_fixture or disc_vs_oracle or rvq or argmin or codes or kmeans" > $O/fft_tests.log 2>&1 || rc=$?
echo "rc=$rc" >> $O/fft_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
VARIANTS="all: nofft:ENCX_FFT=0 norb:ENCX_RESBLOCK=0" ROUNDS=2 BENCH_ARGS="--steps 20" bash tools/gpu_bench_ab.sh > $O/ab.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-graphs > $O/gan_eager.json 2> $O/gan_eager.err || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --config gen > $O/gen.json 2> $O/gen.err || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --no-cpu-baseline --config 48k > $O/48k.json 2> $O/48k.err || exit $?
ENCX_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --no-roofline > $O/rehearse2.json 2> $O/rehearse2.err || exit $?

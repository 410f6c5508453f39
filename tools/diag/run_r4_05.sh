# fused residual block + graphs at world 2: targeted GPU tests (round 4)
O=gpurun_out/r4_05
mkdir -p $O
rc=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread -s -k "resblock" > $O/rb.log 2>&1 || rc=$?
echo "rc=$rc" >> $O/rb.log
if [ $rc -gt 1 ]; then exit $rc; fi
rc=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_train_state.py -x -v --timeout 400 --timeout-method thread -s > $O/model.log 2>&1 || rc=$?
echo "rc=$rc" >> $O/model.log
if [ $rc -gt 1 ]; then exit $rc; fi
rc=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_dp.py tests/test_gpu_dp_full.py -x -v --timeout 800 --timeout-method thread -s > $O/dp.log 2>&1 || rc=$?
echo "rc=$rc" >> $O/dp.log

# tools/diag: HIP-graph replay drift experiments (round 4), logs under gpurun_out/r4_02
#   e1  world 1, segmented step, with a concurrent GPU process (gpu_noise.py)
#   e2  2 ranks on one GPU (gloo), graphs allowed at world 2 (ENCX_DP_GRAPHS=1)
#   e3  e2 with a device sync after every graph replay
#   e4  e2 with HIP's graph packet capture off
set -e
O=gpurun_out/r4_02
mkdir -p $O
# the Conv2d kernels first (new 8-wave weight grad, scheduled dgrad loads); a failed assertion
# (rc 1) continues, anything else (a fault, a timeout) stops here
rc=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_disc.py -x -q --timeout 300 --timeout-method thread -k "conv2d_vs_torch or full_size or disc_vs_oracle" > $O/disc_tests.log 2>&1 || rc=$?
echo "disc tests rc=$rc" >> $O/disc_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/diag/gpu_noise.py --seconds 150 > $O/noise.log 2>&1 &
NP=$!
sleep 15
timeout -k 10 200 python -u tools/diag/graph_repro.py --seg > $O/e1.log 2>&1
wait $NP
ENCX_DP_GRAPHS=1 timeout -k 10 300 python -u tools/diag/dp_graph_diff.py > $O/e2.log 2>&1
ENCX_DP_GRAPHS=1 DP_RSYNC=1 timeout -k 10 300 python -u tools/diag/dp_graph_diff.py > $O/e3.log 2>&1
ENCX_DP_GRAPHS=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 python -u tools/diag/dp_graph_diff.py > $O/e4.log 2>&1
timeout -k 10 300 python -u tools/diag/enc48k_grads.py > $O/enc48k.log 2>&1

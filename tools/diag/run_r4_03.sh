set -e
O=gpurun_out/r4_03
mkdir -p $O
# drift with the round-3 kernels (one-wave weight grad, unscheduled dgrad loads)?
ENCX_DP_GRAPHS=1 ENCX_WGR_WGS=0 ENCX_DGR_VARIANT=4 timeout -k 10 300 python -u tools/diag/dp_graph_diff.py > $O/old_both.log 2>&1
ENCX_DP_GRAPHS=1 ENCX_WGR_WGS=0 timeout -k 10 300 python -u tools/diag/dp_graph_diff.py > $O/old_wgr.log 2>&1
ENCX_DP_GRAPHS=1 ENCX_DGR_VARIANT=4 timeout -k 10 300 python -u tools/diag/dp_graph_diff.py > $O/old_dgr.log 2>&1
VARIANTS="new: oldwg:ENCX_WGR_WGS=0 olddg:ENCX_DGR_VARIANT=4 oldboth:ENCX_WGR_WGS=0,ENCX_DGR_VARIANT=4" ROUNDS=2 BENCH_ARGS="--steps 20" bash tools/gpu_bench_ab.sh > $O/ab.txt 2>&1
rc=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_48k.py tests/test_gpu_dp_full.py -x -v --timeout 600 --timeout-method thread -s > $O/tests.log 2>&1 || rc=$?
echo "tests rc=$rc" >> $O/tests.log

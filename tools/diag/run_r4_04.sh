# round-3 code (git worktree r3wt at bf572e4, graph gate removed): does its world-2 graph drift
# reproduce on today's boxes? Then the config-5 rank-local decomposition test at HEAD.
set -e
O=gpurun_out/r4_04
mkdir -p $O
timeout -k 10 300 python -u r3wt/tools/diag/dp_graph_diff.py > $O/r3_a.log 2>&1
timeout -k 10 300 python -u r3wt/tools/diag/dp_graph_diff.py > $O/r3_b.log 2>&1
rc=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp_full.py -x -v --timeout 500 --timeout-method thread -s -k "decomposition" > $O/tests.log 2>&1 || rc=$?
echo "tests rc=$rc" >> $O/tests.log

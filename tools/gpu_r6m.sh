#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out
export ENCX_LIB=${ENCX_LIB:-encodec-pytorch_amd/stage/r6j.so}
step() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log; case $rc in 124|134|137|139) exit $rc;; esac; [ $rc -ge 128 ] && exit $rc; return 0; }
ENCX_CONV2=1 step d48_1 200 python -u tools/diag/fwd2_48k_diag.py
ENCX_CONV2=0 step d48_0 200 python -u tools/diag/fwd2_48k_diag.py

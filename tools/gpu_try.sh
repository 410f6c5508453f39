#!/bin/bash
# Submit one gpurun command, re-submitting only when the pool reports an infrastructure-side
# transient (no box was acquired and nothing ran). Any run that reached the box ends the loop.
# usage: tools/gpu_try.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && ! grep -q "status=ok" "$LOG"; then
    echo "attempt $i: transient (rc=$rc), waiting" >> "$LOG.tries"
    sleep 100
    continue
  fi
  exit $rc
done
exit 3

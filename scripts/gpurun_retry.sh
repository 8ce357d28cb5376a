#!/bin/bash
# Acquire-retry wrapper for gpurun: re-submits ONLY when gpurun reports that no box / slot was
# available or the box failed while being prepared (nothing ran, nothing charged); any run that
# actually executed is never repeated.   usage: scripts/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; t=$2; cmd=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log"; then
    echo "attempt $i: transient (rc=$rc), retrying" >> "$log.attempts"
    sleep 90
    continue
  fi
  exit $rc
done
exit $rc

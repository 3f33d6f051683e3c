#!/bin/bash
# Submit ONE gpurun command, re-submitting only while the pool reports no free box / slot
# (exit 3, or a "transient" status: nothing ran, nothing was charged).  Any other outcome --
# success or a failure of the command itself -- ends the script (no retry of a GPU step).
#   scripts/gpurun_when_free.sh <log> <timeout_s> '<command>'
log=$1; lim=$2; cmd=$3
for attempt in 1 2 3 4 5 6 7 8; do
  timeout $((lim + 1500)) /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then
    echo "attempt $attempt: no box (rc $rc), waiting" >> "$log.tries"
    sleep 240
    continue
  fi
  echo "attempt $attempt: rc $rc" >> "$log.tries"
  exit $rc
done
exit 3

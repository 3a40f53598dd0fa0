#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool reports that no box
# or slot was free (status=transient, nothing ran, nothing charged).  A call
# that ran -- whatever its exit status -- is never re-submitted.
#   bash scripts/gpurun_when_free.sh <timeout-s> <log> '<command>'
T=$1; LOG=$2; CMD=$3
for attempt in $(seq 1 ${GPURUN_ATTEMPTS:-30}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" && grep -qE "run (0.0s|Nones)" "$LOG"; then
    echo "attempt $attempt: no box free, waiting" >> "$LOG.attempts"
    sleep ${GPURUN_WAIT:-200}
    continue
  fi
  exit $rc
done
exit 3

#!/bin/bash
# Re-submit a gpurun call only while the pool reports "no box / transient" (exit 3).
# Any other outcome (including failures of the command itself) is final.
# usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  echo "[retry-wrapper] attempt $i rc=$rc" >> "$LOG"
  if [ $rc -ne 3 ]; then exit $rc; fi
  sleep 45
done
exit 3

#!/bin/bash
# Retry a gpurun call only when the infrastructure reports a transient failure
# (box lost during preparation / backoff); a command that ran is never retried.
# usage: scripts/gpurun_retry.sh <timeout_s> <log> '<command>'
T=$1; LOG=$2; CMD=$3
for i in 1 2 3 4; do
  timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  if grep -q "status=transient\|backing off\|no box" "$LOG"; then
    sleep 75
    continue
  fi
  break
done
tail -3 "$LOG"

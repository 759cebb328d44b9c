#!/bin/bash
# Retry a gpurun call ONLY while the pool reports "no box free" (exit 3), a transient
# infrastructure status (box lost while being prepared: nothing ran, nothing charged) or an
# infrastructure back-off (nothing ran, nothing charged).  Any other exit, including
# failures of the command itself, ends the loop.
# usage: tools/gpu_try.sh <timeout-s> <max-tries> '<command>'
T=$1; N=$2; CMD=$3
LOG=$(mktemp)
for i in $(seq 1 $N); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" 2>&1 | tee "$LOG"
  rc=${PIPESTATUS[0]}
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG" || { [ $rc -eq 2 ] && grep -q "backing off" "$LOG"; }; then
    sleep 120
    continue
  fi
  rm -f "$LOG"
  exit $rc
done
rm -f "$LOG"
exit 3

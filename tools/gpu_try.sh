#!/bin/bash
# Retry a gpurun call ONLY while the pool reports "no box free" (exit 3: nothing ran,
# nothing charged).  Any other exit (including failures of the command) ends the loop.
# usage: tools/gpu_try.sh <timeout-s> <max-tries> '<command>'
T=$1; N=$2; CMD=$3
for i in $(seq 1 $N); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3

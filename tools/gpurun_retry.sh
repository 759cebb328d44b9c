#!/bin/bash
# Retry a gpurun call while the pool has no free slot/box (gpurun exit 3 / "transient": nothing ran,
# nothing was charged).  Any other outcome -- success or a failure on the box -- is returned as is.
# usage: tools/gpurun_retry.sh <out file> <timeout s> <command>
OUT=$1; TMO=$2; shift 2
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$@" > "$OUT" 2>&1
  rc=$?
  if grep -q "status=transient" "$OUT" && [ $rc -ne 0 ]; then sleep 240; continue; fi
  exit $rc
done
exit 3

#!/bin/bash
# Same-box ABAB of LVC-block phase probes: tools/gpu_probe_ab.sh <tag> <probe A> <probe B> [args]
# (each probe a tools/bin/lvc_probe* binary; args e.g. "256 384 1" = the final block)
set -e
TAG=$1; A=$2; B=$3; shift 3
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
for rep in 1 2; do
  for p in $A $B; do
    timeout -k 10 120 $p "$@" > $O/$(basename $p)_$rep.txt 2>&1
    echo "[$(basename $p) $rep] $(head -1 $O/$(basename $p)_$rep.txt)"
  done
done

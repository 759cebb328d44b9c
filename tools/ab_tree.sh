#!/bin/bash
# Same-box ABAB of the working tree against a snapshot of an earlier tree's host code (tools/bin/prev:
# `git archive <rev> bench.py prodiff_amd include oracle` plus a library), for host-side (Python) changes
# that a library swap cannot A/B.  One job at a time (--overlap 1).
# usage (GPU box): tools/ab_tree.sh <tag> <config> [<config> ...]
set -e
T=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$T; mkdir -p $O
for c in "$@"; do for rep in 1 2; do for side in prev now; do
  d=$R; [ $side = prev ] && d=$R/tools/bin/prev
  (cd $d && timeout -k 10 300 python -u bench.py --config $c --cpu-frames 0 --overlap 1 > $O/${c}_${side}_$rep.json 2> $O/${c}_${side}_$rep.err)
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" $O/${c}_${side}_$rep.json "$c $side $rep"
done; done; done

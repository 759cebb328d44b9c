#!/bin/bash
# Round-over-round on ONE box: the round-4 tree (tools/bin/r04: `git archive 09f8fa7 bench.py prodiff_amd
# include oracle`, its library built there) against the working tree, ABAB per config.
# usage (GPU box): tools/gpu_r04_vs_now.sh <tag> <config> [<config> ...]
# NOW_ARGS: extra bench.py arguments for the working tree only (e.g. "--overlap 1": one job at a
# time, as round 4's bench ran)
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
for c in "$@"; do
  for rep in 1 2; do
    for side in r04 now; do
      d=$R; extra="$NOW_ARGS"; [ $side = r04 ] && d=$R/tools/bin/r04 && extra=""
      (cd $d && timeout -k 10 300 python -u bench.py --config $c --cpu-frames 0 $extra > $O/${c}_${side}_$rep.json 2> $O/${c}_${side}_$rep.err)
      python - $O/${c}_${side}_$rep.json "$c $side $rep" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {t: v["avg_us"] for t, v in d["kernels"].items() if v["ms_total"] > 0.2}
print(f"[{sys.argv[2]}] {d['ms_per_step']} ms/step", k)
PY
    done
  done
done

#!/bin/bash
# Same-box A/B of fd_set_option settings: one C3 bench line per argument ("" = defaults), e.g.
#   tools/gpu_fdopt_ab.sh <tag> "" "kp_chunk=4" "" "kp_chunk=4"
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
i=0
for o in "$@"; do
  i=$((i+1))
  args=""; for kv in $o; do args="$args --fd-opt $kv"; done
  timeout -k 10 300 python -u bench.py --cpu-frames 0 $args > $O/bench_$i.json 2> $O/bench_$i.err
  python - "$o" $O/bench_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {t: v["avg_us"] for t, v in d["kernels"].items() if v["ms_total"] > 0.2}
print(f"[{sys.argv[1]}] {d['ms_per_step']} ms/step", k)
PY
done

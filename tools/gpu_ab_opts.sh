#!/bin/bash
# C3 bench A/B over bench.py option sets (one line each), e.g. tools/gpu_ab_opts.sh <tag> "" "--fd-opt kp_side=1"
set -o pipefail
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
i=0
for opts in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --cpu-frames 0 $opts > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
  python - "$opts" $O/bench_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {t: v["avg_us"] for t, v in d["kernels"].items() if v["ms_total"] > 0.2}
print(f"[{sys.argv[1]}] {d['ms_per_step']} ms/step", k)
PY
done

#!/bin/bash
# A/B the bench under several env settings (one line each), e.g.
#   tools/ab_bench.sh <tag> "" "PRODIFF_LVC_PF=1" "PRODIFF_LVC_TS=256"
# Optional: AB_TESTS=<pytest -k expr> runs those bf16 tests under every setting first;
# BENCH_ARGS=<extra bench.py arguments> (e.g. "--config C5").
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
i=0
for envs in "$@"; do
  i=$((i+1))
  if [ -n "$AB_TESTS" ]; then
    env $envs timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "$AB_TESTS" > $O/tests_$i.log 2>&1
    echo "[$envs] $(tail -1 $O/tests_$i.log)"
  fi
  env $envs timeout -k 10 300 python -u bench.py --cpu-frames 0 $BENCH_ARGS > $O/bench_$i.json 2> $O/bench_$i.err
  python - "$envs" $O/bench_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {t: v["avg_us"] for t, v in d["kernels"].items() if v["ms_total"] > 0.2}
print(f"[{sys.argv[1]}] {d['ms_per_step']} ms/step", k)
PY
done

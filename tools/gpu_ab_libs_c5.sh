#!/bin/bash
# C5 bench A/B over library builds in ab/ (one line each): tools/gpu_ab_libs_c5.sh <tag> lib1 lib2 ...
set -o pipefail
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
for lib in "" "$@" ""; do
  if [ -n "$lib" ]; then export PRODIFF_HIP_LIB=$GRAFT_REPO_ROOT/ab/$lib; else unset PRODIFF_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --config C5 --cpu-frames 0 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python - "$lib" $O/b.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {t: (v["avg_us"], v["tflops"]) for t, v in d["kernels"].items() if t.startswith("nsf_res")}
print(f"[{sys.argv[1]}] {d['ms_per_step']} ms/step", k)
PY
done

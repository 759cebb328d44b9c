#!/bin/bash
# Same-box A/B over library builds and option sets: each argument is "<lib or ->|<bench args>"
# ("-" = the in-tree library), one C3 bench line each, e.g.
#   tools/gpu_ab_libs.sh <tag> "-|" "tools/bin/lib_scalar.so|" "-|--fd-opt lvc_prio=1"
# AB_TESTS=<pytest -k expr> first runs those tests/test_gpu_bf16.py cases under every library.
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
i=0
for spec in "$@"; do
  i=$((i+1))
  lib=${spec%%|*}; args=${spec#*|}
  [ "$lib" = "-" ] && lib=$R/prodiff_amd/libprodiff_hip.so
  if [ -n "$AB_TESTS" ]; then
    PRODIFF_ALLOW_VARIANT=1 PRODIFF_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "$AB_TESTS" > $O/tests_$i.log 2>&1
    echo "[$spec] $(tail -1 $O/tests_$i.log)"
  fi
  PRODIFF_ALLOW_VARIANT=1 PRODIFF_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --cpu-frames 0 $args > $O/bench_$i.json 2> $O/bench_$i.err
  python - "$spec" $O/bench_$i.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {t: v["avg_us"] for t, v in d["kernels"].items() if v["ms_total"] > 0.2}
print(f"[{sys.argv[1]}] {d['ms_per_step']} ms/step", k)
PY
done

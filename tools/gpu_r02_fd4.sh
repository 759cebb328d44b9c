#!/bin/bash
# FastDiff bf16 tests + C3 bench A/B against the previous library (ab/libprodiff_hip_prev.so)
set -o pipefail
O=gpurun_out/r02_fd4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -k "fastdiff or c3" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new old new old; do
  if [ $v = old ]; then export PRODIFF_HIP_LIB=$GRAFT_REPO_ROOT/ab/libprodiff_hip_prev.so; else unset PRODIFF_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --cpu-frames 0 > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python - $v $O/bench_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {t: v["avg_us"] for t, v in d["kernels"].items() if v["ms_total"] > 0.2}
print(f"[{sys.argv[1]}] {d['ms_per_step']} ms/step", k)
PY
done

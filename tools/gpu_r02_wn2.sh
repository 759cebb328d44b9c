#!/bin/bash
# Two-kernel WaveNet layer (GATE + RESSKIP): bf16 tests, C3/C4 bench A/B against the fused kernel
set -o pipefail
O=gpurun_out/r02_wn2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 200 \
  --timeout-method thread -k "wavenet or prodiff or c3_full or c5_full" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "BF16ERR|passed|failed" $O/tests.log | tail -30
for cfg in C3 C4; do
  timeout -k 10 200 python -u bench.py --config $cfg --cpu-frames 0 > $O/bench_${cfg}_new.json 2> $O/bench_${cfg}_new.err || exit 1
  timeout -k 10 200 python -u bench.py --config $cfg --cpu-frames 0 --wn-opt layer=0 > $O/bench_${cfg}_l0.json 2> $O/bench_${cfg}_l0.err || exit 1
done
for f in $O/bench_*.json; do python - $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {t: (v["launches"], v["avg_us"], v["tflops"]) for t, v in d["kernels"].items() if t.startswith("wn")}
print(sys.argv[1], d["ms_per_step"], "ms/step", d["value"], k)
PY
done

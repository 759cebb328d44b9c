#!/bin/bash
# condition stage: GPU tests + timings (round 2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_cond.py tests/test_ckpt.py -m gpu -s > gpurun_out/cond_tests.log 2>&1 || exit 1
for cfg in "1 120 fp32" "1 120 bf16" "8 120 bf16" "32 120 bf16"; do
  set -- $cfg
  timeout -k 10 120 python tools/bench_cond.py --batch $1 --tokens $2 --dtype $3 >> gpurun_out/cond_bench.jsonl 2>> gpurun_out/cond_bench.err || exit 1
done

#!/bin/bash
# full GPU suite after the split-K GEMM change + condition-stage timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -s > gpurun_out/gpu_all.log 2>&1 || exit 1
rm -f gpurun_out/cond_bench2.jsonl
for cfg in "1 120 fp32" "1 120 bf16" "8 120 bf16" "32 120 bf16"; do
  set -- $cfg
  timeout -k 10 120 python tools/bench_cond.py --batch $1 --tokens $2 --dtype $3 >> gpurun_out/cond_bench2.jsonl 2>> gpurun_out/cond_bench.err || exit 1
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 1

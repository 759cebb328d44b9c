#!/bin/bash
# fp32 split-K WaveNet (C2) + full GPU suite + C2/C3/C5 lines
set -o pipefail
mkdir -p gpurun_out/r02c2
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r02c2/gpu_all.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config C2 --steps 20 --warmup 3 > gpurun_out/r02c2/bench_c2.json 2> gpurun_out/r02c2/err.log || exit 1
timeout -k 10 300 python bench.py --config C2 --no-graph --steps 10 --warmup 3 --cpu-frames 0 > gpurun_out/r02c2/bench_c2_eager.json 2>> gpurun_out/r02c2/err.log || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-frames 0 > gpurun_out/r02c2/bench_c3.json 2>> gpurun_out/r02c2/err.log || exit 1

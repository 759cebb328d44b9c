#!/bin/bash
# C5 (SVS) pipeline: GPU test + bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_cond.py -m gpu -k svs -s > gpurun_out/c5_test.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config C5 --steps 3 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || exit 1

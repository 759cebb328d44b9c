#!/bin/bash
# NSF windowed conv: tests + NSF bench A/B + C5 line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_nsf.py -m gpu -s > gpurun_out/nsf_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 > gpurun_out/bench_c5_wconv.json 2> gpurun_out/bench_c5.err || exit 1

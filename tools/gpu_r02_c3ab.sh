#!/bin/bash
# C3 check after a FastDiff kernel change: bf16 + fullsize GPU tests, then two bench lines
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bf16.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-frames 0 > $O/bench_a.json 2> $O/err.log || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-frames 0 > $O/bench_b.json 2>> $O/err.log || exit 1
timeout -k 10 300 python bench.py --config C2 --steps 20 --warmup 3 --cpu-frames 0 > $O/bench_c2.json 2>> $O/err.log || exit 1

#!/bin/bash
# two-kernel WaveNet layer (option layer=1): bf16 goldens for every layer mode + a forced layer=1 C3 bench
set -o pipefail
O=gpurun_out/r02_wn3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "wavenet or prodiff" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "BF16ERR|passed|failed" $O/tests.log | tail -14
timeout -k 10 200 python -u bench.py --config C3 --cpu-frames 0 --wn-opt layer=1 > $O/bench_C3_l1.json 2> $O/bench_C3_l1.err || exit 1
timeout -k 10 200 python -u bench.py --config C3 --cpu-frames 0 > $O/bench_C3.json 2> $O/bench_C3.err || exit 1
tail -c 300 $O/bench_C3_l1.json; tail -c 300 $O/bench_C3.json

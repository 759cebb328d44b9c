#!/bin/bash
set -o pipefail
O=gpurun_out/r02_chunk
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fastdiff" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
tools/gpu_ab_opts.sh r02_chunk_ab "" "--fd-opt kp_chunk=4" "--fd-opt kp_chunk=2" "" "--fd-opt kp_chunk=4" "--fd-opt kp_chunk=1"

#!/bin/bash
# r04 step 8: WaveNet stack, branch-free LVC gate, kp bias-in-accumulator, NSF ResBlock pair:
# parity, then same-box A/Bs for C3 and C5.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bf16.py \
  tests/test_gpu_draws.py tests/test_gpu_nsf.py "tests/test_gpu_fullsize.py::test_c3_full_bf16_vs_fp32" \
  "tests/test_gpu_fullsize.py::test_c5_full_bf16_vs_fp32" > $O/tests.log 2>&1
tail -3 $O/tests.log
tools/gpu_ab_libs.sh $TAG/c3 'tools/bin/lib_base.so|' '-|' '-|--wn-opt stack=10' '-|--wn-opt stack=7' \
  'tools/bin/lib_base.so|' '-|' '-|--wn-opt stack=10' '-|--wn-opt stack=7'
BENCH_ARGS_C5="--config C5"
tools/gpu_ab_libs.sh $TAG/c5 'tools/bin/lib_base.so|--config C5' '-|--config C5 --nsf-opt pair=0' '-|--config C5' \
  '-|--config C5 --wn-opt stack=10' 'tools/bin/lib_base.so|--config C5' '-|--config C5 --nsf-opt pair=0' '-|--config C5'

#!/bin/bash
# r04 step 7: 8-wave WaveNet stack kernel, branch-free LVC gate (PF), kp bias-in-accumulator.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bf16.py \
  tests/test_gpu_draws.py "tests/test_gpu_fullsize.py::test_c3_full_bf16_vs_fp32" > $O/tests.log 2>&1
tail -3 $O/tests.log
grep -h "BF16ERR" $O/tests.log | tail -6
tools/gpu_ab_libs.sh $TAG/ab 'tools/bin/lib_base.so|' '-|' '-|--wn-opt stack=10' '-|--wn-opt stack=7' \
  'tools/bin/lib_base.so|' '-|' '-|--wn-opt stack=10' '-|--wn-opt stack=7'

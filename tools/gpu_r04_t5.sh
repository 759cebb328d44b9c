#!/bin/bash
# r04 step 5: WaveNet stack kernel + pre-scaled kp weights: parity, then a same-box A/B.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bf16.py \
  -k "stack_bitexact or schedule_variants or fastdiff_sample_bf16 or kp_chunk or lvc_block_bf16 or wavenet_bf16" \
  "tests/test_gpu_fullsize.py::test_c3_full_bf16_vs_fp32" > $O/tests.log 2>&1
tail -3 $O/tests.log
grep -h "BF16ERR" $O/tests.log | tail -8
tools/gpu_ab_libs.sh $TAG/ab 'tools/bin/lib_base.so|' '-|' '-|--wn-opt stack=10' '-|--wn-opt stack=5' '-|--wn-opt stack=4' \
  'tools/bin/lib_base.so|' '-|' '-|--wn-opt stack=10' '-|--wn-opt stack=5'

#!/bin/bash
# r04 step 12: WaveNet stack launches with the fused input projection / sampler output stage
# (PD_WN_OPT_STACK_FUSE) and rows per block (PD_WN_OPT_STACK_RO): parity + same-box A/B (C3, C5).
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bf16.py \
  -k "stack or prodiff or wavenet" tests/test_gpu_parity.py tests/test_gpu_draws.py \
  "tests/test_gpu_fullsize.py::test_c3_full_bf16_vs_fp32" "tests/test_gpu_fullsize.py::test_c2_prodiff_fullsize_fp32" \
  > $O/tests.log 2>&1
tail -3 $O/tests.log
tools/gpu_ab_libs.sh $TAG/c3 'tools/bin/lib_af3e369.so|' '-|' '-|--wn-opt stack_fuse=0' \
  'tools/bin/lib_af3e369.so|' '-|' '-|--wn-opt stack_fuse=0'
tools/gpu_ab_libs.sh $TAG/c5 'tools/bin/lib_af3e369.so|--config C5' '-|--config C5'

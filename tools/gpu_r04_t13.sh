#!/bin/bash
# r04 step 13: fp32 residual layers on wn_f32_layer_kernel (PD_WN_OPT_F32_LAYER, C2) and the fused
# stack output stage at M = 128 (C5): parity + same-box A/B.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_bf16.py -k "not lvc and not fastdiff" "tests/test_gpu_fullsize.py::test_c2_prodiff_fullsize_fp32" \
  tests/test_gpu_draws.py > $O/tests.log 2>&1
tail -3 $O/tests.log
tools/gpu_ab_libs.sh $TAG/c2 'tools/bin/lib_af3e369.so|--config C2' '-|--config C2' '-|--config C2 --wn-opt f32_layer=0' \
  'tools/bin/lib_af3e369.so|--config C2' '-|--config C2'
tools/gpu_ab_libs.sh $TAG/c5 'tools/bin/lib_af3e369.so|--config C5' '-|--config C5' '-|--config C5 --wn-opt stack_fuse=0' \
  'tools/bin/lib_af3e369.so|--config C5' '-|--config C5'

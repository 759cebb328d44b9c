#!/bin/bash
# r04 step 26: NSF ResBlock pair kernel with xt written over x's window after a barrier (one window per
# block: 2 blocks per CU at C = 128) (lib_pairx) vs lib_head: NSF parity, C5 A/B.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
PRODIFF_HIP_LIB=$R/tools/bin/lib_pairx.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_nsf.py tests/test_gpu_draws.py "tests/test_gpu_fullsize.py::test_c5_full_bf16_vs_fp32" > $O/tests.log 2>&1
tail -1 $O/tests.log
tools/gpu_ab_libs.sh $TAG/c5 'tools/bin/lib_head.so|--config C5' 'tools/bin/lib_pairx.so|--config C5' \
  'tools/bin/lib_head.so|--config C5' 'tools/bin/lib_pairx.so|--config C5'

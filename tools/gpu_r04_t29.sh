#!/bin/bash
# r04 step 29: the C = 32 NSF pair kernel on 480-row blocks (FMO 15: c1 recomputes 1 row tile in 16
# instead of 1 in 8, the window halo is amortised over twice the rows) (lib_f15) vs lib_head (224-row
# blocks): NSF parity, C5 A/B.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
PRODIFF_HIP_LIB=$R/tools/bin/lib_f15.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_nsf.py tests/test_gpu_draws.py "tests/test_gpu_fullsize.py::test_c5_full_bf16_vs_fp32" > $O/tests_f15.log 2>&1
tail -1 $O/tests_f15.log
tools/gpu_ab_libs.sh $TAG/c5 'tools/bin/lib_head.so|--config C5' 'tools/bin/lib_f15.so|--config C5' \
  'tools/bin/lib_head.so|--config C5' 'tools/bin/lib_f15.so|--config C5'

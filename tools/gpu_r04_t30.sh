#!/bin/bash
# r04 step 30: the C = 64 NSF pair kernel on 256-row blocks (FMO 8: c1 recomputes 1 row tile in 9
# instead of 1 in 5, the halo amortised over twice the rows) (lib_f64) vs lib_head (128-row
# blocks): NSF parity, C5 A/B.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
PRODIFF_HIP_LIB=$R/tools/bin/lib_f64.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_nsf.py tests/test_gpu_draws.py "tests/test_gpu_fullsize.py::test_c5_full_bf16_vs_fp32" > $O/tests_f64.log 2>&1
tail -1 $O/tests_f64.log
tools/gpu_ab_libs.sh $TAG/c5 'tools/bin/lib_head.so|--config C5' 'tools/bin/lib_f64.so|--config C5' \
  'tools/bin/lib_head.so|--config C5' 'tools/bin/lib_f64.so|--config C5'

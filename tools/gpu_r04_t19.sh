#!/bin/bash
# r04 step 19: NSF ResBlock pair kernel at C = 32 (+ the DBlock changes of step 18), lib_wt: parity and
# same-box C5 A/B vs the committed library.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
PRODIFF_HIP_LIB=$R/tools/bin/lib_wt.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_nsf.py "tests/test_gpu_fullsize.py::test_c5_full_bf16_vs_fp32" > $O/tests.log 2>&1
tail -2 $O/tests.log
tools/gpu_ab_libs.sh $TAG/c5 'tools/bin/lib_bc2488e.so|--config C5' 'tools/bin/lib_wt.so|--config C5' \
  'tools/bin/lib_bc2488e.so|--config C5' 'tools/bin/lib_wt.so|--config C5'

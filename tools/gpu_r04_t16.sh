#!/bin/bash
# r04 step 16: fp32 layer / tail kernels with branch-free operand loads: C2.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "fp32 or wavenet or prodiff" "tests/test_gpu_fullsize.py::test_c2_prodiff_fullsize_fp32" > $O/tests.log 2>&1
tail -2 $O/tests.log
tools/gpu_ab_libs.sh $TAG/c2 'tools/bin/lib_fc71141.so|--config C2' '-|--config C2' 'tools/bin/lib_fc71141.so|--config C2' '-|--config C2'

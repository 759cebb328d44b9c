#!/bin/bash
# r04 step 21: FastDiff prologues without waits at branch joins -- LVC small operands at clamped
# indices, branch-free phase-GEMM weight loads, explicit draws read in the epilogue; kp_hidden biases
# preloaded (lib_fdbf) vs the committed library: parity and same-box C3 A/B.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
PRODIFF_HIP_LIB=$R/tools/bin/lib_fdbf.so timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_bf16.py tests/test_gpu_draws.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1
tail -2 $O/tests.log
tools/gpu_ab_libs.sh $TAG/c3 'tools/bin/lib_7e7b715.so|' 'tools/bin/lib_fdbf.so|' 'tools/bin/lib_7e7b715.so|' 'tools/bin/lib_fdbf.so|'

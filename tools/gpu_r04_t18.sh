#!/bin/bash
# r04 step 18: DBlock with a compile-time audio/x input and unconditional staging stores (lib_dbaud) vs
# the committed library; 256-sample tiles for the hop >= 64 LVC blocks (--fd-opt lvc_ts=256).
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
PRODIFF_HIP_LIB=$R/tools/bin/lib_dbaud.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_bf16.py -k "fastdiff" "tests/test_gpu_fullsize.py::test_c3_full_bf16_vs_fp32" tests/test_gpu_parity.py \
  -k "fastdiff or c3" > $O/tests.log 2>&1
tail -2 $O/tests.log
tools/gpu_ab_libs.sh $TAG/c3 'tools/bin/lib_bc2488e.so|' 'tools/bin/lib_dbaud.so|' '-|--fd-opt lvc_ts=256' \
  'tools/bin/lib_bc2488e.so|' 'tools/bin/lib_dbaud.so|' '-|--fd-opt lvc_ts=256'

#!/bin/bash
# r04 step 23: NSF pair kernel with its residual loads issued before c2's MFMAs and range-checked buffer
# stores (lib_pair) vs lib_kpws: NSF parity, C5 A/B.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
PRODIFF_HIP_LIB=$R/tools/bin/lib_pair.so timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_nsf.py tests/test_gpu_draws.py "tests/test_gpu_fullsize.py::test_c5_full_bf16_vs_fp32" > $O/tests.log 2>&1
tail -2 $O/tests.log
tools/gpu_ab_libs.sh $TAG/c5 'tools/bin/lib_kpws.so|--config C5' 'tools/bin/lib_pair.so|--config C5' \
  'tools/bin/lib_kpws.so|--config C5' 'tools/bin/lib_pair.so|--config C5'

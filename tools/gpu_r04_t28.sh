#!/bin/bash
# r04 step 28: NSF pair kernel -- C = 64 with x and xt side by side again (lib_na64: the one-window
# layout ran C = 64 at 274 -> 294 us while C = 128 / 32 gained), and c1's epilogue with a tile-uniform
# range test and med3 leaky_relu (lib_c1f); vs lib_head: NSF parity, C5 A/B.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
for v in na64 c1f; do
  PRODIFF_HIP_LIB=$R/tools/bin/lib_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    -m gpu tests/test_gpu_nsf.py tests/test_gpu_draws.py "tests/test_gpu_fullsize.py::test_c5_full_bf16_vs_fp32" > $O/tests_$v.log 2>&1
  tail -1 $O/tests_$v.log
done
tools/gpu_ab_libs.sh $TAG/c5 'tools/bin/lib_head.so|--config C5' 'tools/bin/lib_na64.so|--config C5' 'tools/bin/lib_c1f.so|--config C5' \
  'tools/bin/lib_head.so|--config C5' 'tools/bin/lib_na64.so|--config C5' 'tools/bin/lib_c1f.so|--config C5'

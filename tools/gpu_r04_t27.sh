#!/bin/bash
# r04 step 27: C = 256 NSF ResBlock convs on 64-row blocks where a 128-row block's LDS window leaves room
# for one block per CU (lib_w256a) or always (lib_w256b); NSF pair kernel without branches around its
# MFMAs, tile-uniform range tests, med3 leaky_relu and buffer-store epilogue, plus the 16-channel conv with
# compile-time tap pairs (lib_pairv); vs lib_head:
# NSF parity, C5 A/B.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
for v in pairv w256a w256b; do
  PRODIFF_HIP_LIB=$R/tools/bin/lib_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    -m gpu tests/test_gpu_nsf.py tests/test_gpu_draws.py "tests/test_gpu_fullsize.py::test_c5_full_bf16_vs_fp32" > $O/tests_$v.log 2>&1
  tail -1 $O/tests_$v.log
done
tools/gpu_ab_libs.sh $TAG/c5 'tools/bin/lib_head.so|--config C5' 'tools/bin/lib_pairv.so|--config C5' 'tools/bin/lib_w256a.so|--config C5' \
  'tools/bin/lib_w256b.so|--config C5' 'tools/bin/lib_head.so|--config C5' 'tools/bin/lib_pairv.so|--config C5' \
  'tools/bin/lib_w256a.so|--config C5' 'tools/bin/lib_w256b.so|--config C5'

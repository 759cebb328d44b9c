#!/bin/bash
# r04 step 25: DBlock audio window aliased into H1 (40.3 KB LDS) + last-stage weights loaded after
# stage 1 (<= 96 VGPRs): 4 blocks of 5 waves per CU instead of 3 (lib_db4) vs lib_head: FastDiff
# bf16 + full-size tests under lib_db4, C3 A/B.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
PRODIFF_HIP_LIB=$R/tools/bin/lib_db4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  -m gpu tests/test_gpu_bf16.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "fastdiff or c3 or dblock" \
  > $O/tests_db4.log 2>&1
tail -1 $O/tests_db4.log
tools/gpu_ab_libs.sh $TAG/c3 'tools/bin/lib_head.so|' 'tools/bin/lib_db4.so|' 'tools/bin/lib_head.so|' 'tools/bin/lib_db4.so|'

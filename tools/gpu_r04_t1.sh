#!/bin/bash
# r04 step 1: new tests (bf16 draws, RCCL world-1, whole C3 waveform, one-tile-per-wave LVC) and a
# same-box A/B of the LVC tiles-per-wave option.   usage (GPU box): tools/gpu_r04_t1.sh <tag>
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu \
  tests/test_gpu_bf16.py::test_fastdiff_lvc_one_tile_per_wave tests/test_gpu_draws.py tests/test_gpu_rccl.py \
  "tests/test_gpu_fullsize.py::test_c3_slice_fastdiff_fp32" > $O/tests.log 2>&1
tail -3 $O/tests.log
tools/gpu_fdopt_ab.sh $TAG/ab "" "lvc_tpw=1 lvc_pf=0" "lvc_pf=0" "lvc_tpw=1" "" "lvc_tpw=1 lvc_pf=0"

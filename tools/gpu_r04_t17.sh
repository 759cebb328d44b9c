#!/bin/bash
# r04 step 17: hop >= 32 LVC blocks prefetch their audio-rate conditioning rows in the prologue; same-box
# A/B vs the previous commit and vs round 3's library (lib_base).
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bf16.py \
  -k "fastdiff or lvc" "tests/test_gpu_fullsize.py::test_c3_full_bf16_vs_fp32" tests/test_gpu_draws.py > $O/tests.log 2>&1
tail -2 $O/tests.log
tools/gpu_ab_libs.sh $TAG/c3 'tools/bin/lib_bc2488e.so|' '-|' 'tools/bin/lib_base.so|' 'tools/bin/lib_bc2488e.so|' '-|' 'tools/bin/lib_base.so|'

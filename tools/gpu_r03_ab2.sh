#!/bin/bash
# r03: bf16 parity tests, then same-box A/B bench lines: base library (arg 2) vs the tree's, ABAB.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r03_ab2}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_bench.sh ${1:-r03_ab2} "PRODIFF_HIP_LIB=$2" "" "PRODIFF_HIP_LIB=$2" ""

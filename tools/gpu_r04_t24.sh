#!/bin/bash
# r04 step 24: fp32 layer kernel epilogue with preloaded operands and range-checked buffer stores; operand ring
# depth 3 (lib_wfr3) vs 2 (lib_wfr2) vs lib_kpws: fp32 parity, C2 A/B.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
for v in wfr3 wfr2; do
  PRODIFF_HIP_LIB=$R/tools/bin/lib_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    -m gpu tests/test_gpu_parity.py -k "fp32 or wavenet or prodiff" "tests/test_gpu_fullsize.py::test_c2_prodiff_fullsize_fp32" \
    > $O/tests_$v.log 2>&1
  tail -1 $O/tests_$v.log
done
tools/gpu_ab_libs.sh $TAG/c2 'tools/bin/lib_kpws.so|--config C2' 'tools/bin/lib_wfr3.so|--config C2' 'tools/bin/lib_wfr2.so|--config C2' \
  'tools/bin/lib_kpws.so|--config C2' 'tools/bin/lib_wfr3.so|--config C2' 'tools/bin/lib_wfr2.so|--config C2'

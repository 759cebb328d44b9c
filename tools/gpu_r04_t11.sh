#!/bin/bash
# r04 step 11: DBlock tile loop (FD_OPT_DB_NSUB), 6-wave kp_hidden, WN stack rows per block
# (PD_WN_OPT_STACK_RO), fp32 in-kernel split-K (PD_WN_OPT_KSPLIT_FUSED): parity + same-box A/B; C2 kernel trace.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bf16.py \
  -k "nsub or fastdiff_forward or fastdiff_sample_bf16 or stack or kp_chunk" \
  "tests/test_gpu_fullsize.py::test_c3_full_bf16_vs_fp32" tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_c2_prodiff_fullsize_fp32" \
  > $O/tests.log 2>&1
tail -3 $O/tests.log
tools/gpu_ab_libs.sh $TAG/c3 'tools/bin/lib_af3e369.so|' '-|' '-|--fd-opt db_nsub=1' '-|--fd-opt db_nsub=3' \
  '-|--wn-opt stack_ro=32' 'tools/bin/lib_af3e369.so|' '-|' '-|--fd-opt db_nsub=1' '-|--wn-opt stack_ro=32'
tools/gpu_ab_libs.sh $TAG/c2 'tools/bin/lib_af3e369.so|--config C2' '-|--config C2' '-|--config C2 --wn-opt ksplit_fused=0' \
  'tools/bin/lib_af3e369.so|--config C2' '-|--config C2' '-|--config C2 --wn-opt ksplit=256'
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2prof -o c2 -- python3 $R/bench.py --config C2 --steps 20 \
  --warmup 5 --cpu-frames 0 > $O/c2_bench.json 2> $O/c2_bench.err
find $O/c2prof -name "*kernel_stats.csv"

#!/bin/bash
# r04 final measurement set, part <1|2>:
#   1: every -m gpu test, the C3 / C2 / C4-on-1-GPU / C5 bench lines, the C3 and C5 rocprofv3
#      kernel-trace summaries
#   2: FETCH/WRITE PMC passes (C3, C4) on the FastDiff kernels and the SQ passes (C3, C5)
# usage (GPU box): tools/gpu_r04_final.sh <tag> <1|2>
set -e
TAG=$1; PART=$2; RE="lvc_block_bf16_kernel|kp_kernel_bf16"
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
if [ "$PART" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -2 $O/gpu_tests.log
  timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err
  timeout -k 10 300 python -u bench.py --config C2 > $O/bench_c2.json 2> $O/bench_c2.err
  timeout -k 10 300 python -u bench.py --config C4 --cpu-frames 0 > $O/bench_c4_1gpu.json 2> $O/bench_c4.err
  timeout -k 10 300 python -u bench.py --config C5 > $O/bench_c5.json 2> $O/bench_c5.err
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python -u $R/bench.py --cpu-frames 0 --no-kernel-timing > $O/trace.log 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o run --output-format csv -- \
    python -u $R/bench.py --config C5 --cpu-frames 0 --no-kernel-timing > $O/trace_c5.log 2>&1
else
  cd /tmp && export TMPDIR=/tmp
  for pmc in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$RE" -d $O/pmc_$pmc -o run --output-format csv -- \
      python -u $R/bench.py --steps 2 --warmup 1 --cpu-frames 0 --no-kernel-timing > $O/pmc_$pmc.log 2>&1
    timeout -s KILL 180 rocprofv3 --pmc $pmc --kernel-include-regex "$RE" -d $O/c4/pmc_$pmc -o run --output-format csv -- \
      python -u $R/bench.py --config C4 --steps 2 --warmup 1 --cpu-frames 0 --no-kernel-timing > $O/c4_pmc_$pmc.log 2>&1
  done
  cd $R
  timeout -k 10 400 tools/pmc_sq.sh $TAG/c3 "lvc_block_bf16|kp_kernel_bf16|wn_stack_bf16|dblock_bf16|kp_hidden_bf16" --steps 2
  timeout -k 10 400 tools/pmc_sq.sh $TAG/c5 "nsf_|enc_|wn_stack_bf16|wn_layer_bf16" --config C5 --steps 1
fi
echo done

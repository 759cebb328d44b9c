#!/bin/bash
# One gpurun call: GPU parity tests, the default bench line (with cpu_baseline), the
# rocprofv3 kernel-trace summary of the same bench command, and separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) on the dominant kernel.
# usage (on the GPU box): tools/gpu_round.sh <tag> [tests|notests] [kernel-regex]
# Every GPU step has its own time limit; the first failure ends the script.
set -e
TAG=$1; MODE=${2:-tests}; RE=${3:-lvc_block_bf16_kernel|kp_kernel_bf16}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$MODE" = "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
  tail -3 $O/gpu_tests.log
fi
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python -u $R/bench.py --cpu-frames 0 --no-kernel-timing > $O/trace.log 2>&1
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$RE" -d $O/pmc_$pmc -o run --output-format csv -- \
    python -u $R/bench.py --steps 2 --warmup 1 --cpu-frames 0 --no-kernel-timing > $O/pmc_$pmc.log 2>&1
done
echo done

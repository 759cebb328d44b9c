#!/bin/bash
# r04 closing set after the C = 32 pair-block change: every -m gpu test, the C5 and C3 bench lines and
# the C5 rocprofv3 kernel-trace summary.
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --config C5 > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o run --output-format csv -- \
  python -u $R/bench.py --config C5 --cpu-frames 0 --no-kernel-timing > $O/trace_c5.log 2>&1
echo done

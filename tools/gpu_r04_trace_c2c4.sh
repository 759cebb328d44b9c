#!/bin/bash
# r04: rocprofv3 kernel-trace summaries of the C2 (fp32, hipGraph) and C4-on-one-GPU bench commands
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o run --output-format csv -- \
  python -u $R/bench.py --config C2 --cpu-frames 0 --no-kernel-timing > $O/trace_c2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o run --output-format csv -- \
  python -u $R/bench.py --config C4 --cpu-frames 0 --no-kernel-timing > $O/trace_c4.log 2>&1
echo done

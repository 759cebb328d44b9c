#!/bin/bash
# per-kernel-instance timing of the C5 step (rocprofv3 kernel trace)
set -o pipefail
mkdir -p gpurun_out/nsfprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/nsfprof -o c5 -- python3 $GRAFT_REPO_ROOT/bench.py --config C5 --steps 2 --warmup 1 --no-kernel-timing > $GRAFT_REPO_ROOT/gpurun_out/nsfprof/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/nsfprof/bench.err || exit 1

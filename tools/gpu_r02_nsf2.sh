#!/bin/bash
# NSF windowed conv v2 (register ring prefetch, branch-free epilogue): tests + rocprof kernel trace + C5 line
set -o pipefail
mkdir -p gpurun_out/nsfprof10
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_nsf.py -m gpu -s > gpurun_out/nsf_tests10.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/nsfprof10 -o c5 -- python3 $GRAFT_REPO_ROOT/bench.py --config C5 --steps 2 --warmup 1 --no-kernel-timing > $GRAFT_REPO_ROOT/gpurun_out/nsfprof10/bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/nsfprof10/bench.err || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 > gpurun_out/bench_c5_wconv10.json 2> gpurun_out/bench_c5.err || exit 1

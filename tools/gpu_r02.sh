#!/bin/bash
# Round-2 GPU call: every -m gpu test (no -x: collect all bf16 error lines), then the bench
# lines C3 (default), C2 (hipGraph) and C4 on one GPU.  Each GPU step has its own limit.
# usage (on the GPU box): tools/gpu_r02.sh <tag> [tests|notests]
set -e
TAG=$1; MODE=${2:-tests}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$MODE" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rA > $O/gpu_tests.log 2>&1 || echo "TESTS FAILED"
  tail -5 $O/gpu_tests.log
  grep BF16ERR $O/gpu_tests.log | sort | uniq > $O/bf16err.txt || true
fi
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err
cat $O/bench_c3.json
timeout -k 10 300 python -u bench.py --config C2 --steps 20 --warmup 3 > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 300 python -u bench.py --config C2 --steps 20 --warmup 3 --no-graph --cpu-frames 0 > $O/bench_c2_eager.json 2> $O/bench_c2e.err
timeout -k 10 300 python -u bench.py --config C4 --cpu-frames 0 > $O/bench_c4_1gpu.json 2> $O/bench_c4.err
echo done

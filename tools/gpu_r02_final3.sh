#!/bin/bash
# Round-2 (session 2) state: full GPU suite + smoke, C3 line + rocprof + PMC, C5 line + rocprof + PMC, C2 line
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_v4_smoke.log 2>&1
tail -2 gpurun_out/r02_v4_smoke.log
tools/gpu_round.sh r02_v4 tests
tools/gpu_round_c5.sh r02_v4c5
cd $R
timeout -k 10 200 python -u bench.py --config C2 > gpurun_out/r02_v4/bench_c2.json 2> gpurun_out/r02_v4/bench_c2.err
echo all-done

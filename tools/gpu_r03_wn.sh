#!/bin/bash
# r03: WaveNet layer / DBlock changes -- their parity tests, then the C3 bench line and SQ counters
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r03_wn}; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u bench.py --cpu-frames 0 > $O/bench.json 2> $O/bench.err
python -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
if [ -n "$2" ]; then bash tools/pmc_sq.sh $1/sq "$2" && python tools/pmc_sq.py $O/sq > $O/sq_summary.txt; fi

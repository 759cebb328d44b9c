#!/bin/bash
# Round-2 GPU call: streaming-LVC smoke (small cases first), full -m gpu suite, then bench A/B.
# usage (on the GPU box): tools/gpu_r02b.sh <tag>
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -k "stream" -x -v --timeout 120 --timeout-method thread > $O/stream_tests.log 2>&1
tail -3 $O/stream_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log
grep BF16ERR $O/gpu_tests.log | sort | uniq > $O/bf16err.txt || true
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python -u bench.py --cpu-frames 0 --fd-opt lvc_stream=0 > $O/bench_c3_nostream.json 2> $O/bench_c3ns.err
python -c "
import json
for f in ['bench_c3','bench_c3_nostream']:
    d=json.load(open('$O/'+f+'.json')); print(f, d['ms_per_step'], d['value'], {k:v['avg_us'] for k,v in list(d['kernels'].items())[:7]})"
echo done

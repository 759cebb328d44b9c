#!/bin/bash
# stream-kernel iteration: LVC tests, bench A/B (stream vs whole-block), SQ counters of the stream kernel
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --cpu-frames 0 > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python -u bench.py --cpu-frames 0 --fd-opt lvc_stream=0 > $O/bench_c3_nostream.json 2> $O/bench_c3ns.err
python -c "
import json
for f in ['bench_c3','bench_c3_nostream']:
    d=json.load(open('$O/'+f+'.json')); print(f, d['ms_per_step'], d['value'], {k:v['avg_us'] for k,v in list(d['kernels'].items())[:7]})"
tools/pmc_sq.sh $TAG lvc_stream
python tools/pmc_sq.py $O > $O/sq_summary.txt && cat $O/sq_summary.txt
echo done

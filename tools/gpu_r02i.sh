#!/bin/bash
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log
grep BF16ERR $O/tests.log | grep -i "wavenet\|prodiff\|C3" || true
timeout -k 10 300 python -u bench.py --cpu-frames 0 > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python -u bench.py --cpu-frames 0 --wn-opt layer=0 > $O/bench_c3_fusedwn.json 2> $O/bench_c3f.err
timeout -k 10 300 python -u bench.py --cpu-frames 0 --config C4 > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python -u bench.py --cpu-frames 0 --config C4 --wn-opt layer=0 > $O/bench_c4_w0.json 2> $O/bench_c4w0.err
python -c "
import json
for f in ['bench_c3','bench_c3_fusedwn','bench_c4','bench_c4_w0']:
    d=json.load(open('$O/'+f+'.json')); print(f, d['ms_per_step'], d['value'], {k:(v['avg_us'],v['launches'],v['tflops']) for k,v in list(d['kernels'].items())[:9]})"
echo done

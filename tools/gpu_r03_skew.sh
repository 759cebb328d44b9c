#!/bin/bash
# r03: skewed persistent LVC kernel -- parity tests, then C3 bench lines with it on (A) and off (B).
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r03_skew}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 120 --timeout-method thread \
  -k "skew or lvc_block or sample_bf16_oracle" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
grep BF16ERR $O/tests.log | grep skew | tail -12
for v in 1 0; do
  timeout -k 10 200 python -u bench.py --cpu-frames 0 --fd-opt lvc_skew=$v > $O/bench_skew$v.json 2> $O/bench$v.err
  python -c "import json; d=json.load(open('$O/bench_skew$v.json')); print('skew=$v', d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('fd_')})"
done

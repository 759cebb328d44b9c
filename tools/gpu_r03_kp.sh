#!/bin/bash
# r03: kernel-predictor K stores -- bf16 parity tests, then C3 bench lines per store variant / timing probe.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r03_kp}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in "kp_nt=1" "kp_nt=0" "kp_probe=1" "kp_probe=2"; do
  timeout -k 10 200 python -u bench.py --cpu-frames 0 --fd-opt $v > $O/bench_$v.json 2> $O/bench_$v.err
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('fd_')})"
done

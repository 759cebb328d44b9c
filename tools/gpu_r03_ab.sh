set -e
timeout -k 10 120 tools/bin/skew_probe > gpurun_out/skew_probe2.txt 2>&1; cat gpurun_out/skew_probe2.txt
for v in 1 0; do
  timeout -k 10 200 python -u bench.py --cpu-frames 0 --fd-opt lvc_skew=$v > gpurun_out/r03_ab_skew$v.json 2> /dev/null
  python -c "import json; d=json.load(open('gpurun_out/r03_ab_skew$v.json')); print('skew=$v', d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items() if k.startswith('fd_')})"
done

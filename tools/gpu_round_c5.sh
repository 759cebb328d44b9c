#!/bin/bash
# C5 (SVS) bench line, its rocprofv3 kernel-trace summary, and FETCH/WRITE passes on the
# windowed NSF convs.  usage (on the GPU box): tools/gpu_round_c5.sh <tag>
set -e
TAG=$1; RE=${2:-nsf_wconv_kernel}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --config C5 > $O/bench_c5.json 2> $O/bench_c5.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python -u $R/bench.py --config C5 --cpu-frames 0 --no-kernel-timing > $O/trace.log 2>&1
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$RE" -d $O/pmc_$pmc -o run --output-format csv -- \
    python -u $R/bench.py --config C5 --steps 2 --warmup 1 --cpu-frames 0 --no-kernel-timing > $O/pmc_$pmc.log 2>&1
done
echo done

#!/bin/bash
# r03 final measurement set (no tests): C3 / C2 / C4-on-1-GPU / C5 bench lines, the C3 rocprofv3
# kernel-trace summary, and FETCH/WRITE PMC passes for C3 and C4 on the FastDiff kernels.
# usage (GPU box): tools/gpu_r03_final.sh <tag>
set -e
TAG=$1; RE="lvc_block_bf16_kernel|kp_kernel_bf16"
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python -u bench.py --config C2 > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 300 python -u bench.py --config C4 --cpu-frames 0 > $O/bench_c4_1gpu.json 2> $O/bench_c4.err
timeout -k 10 300 python -u bench.py --config C5 > $O/bench_c5.json 2> $O/bench_c5.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python -u $R/bench.py --cpu-frames 0 --no-kernel-timing > $O/trace.log 2>&1
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$RE" -d $O/pmc_$pmc -o run --output-format csv -- \
    python -u $R/bench.py --steps 2 --warmup 1 --cpu-frames 0 --no-kernel-timing > $O/pmc_$pmc.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc $pmc --kernel-include-regex "$RE" -d $O/c4/pmc_$pmc -o run --output-format csv -- \
    python -u $R/bench.py --config C4 --steps 2 --warmup 1 --cpu-frames 0 --no-kernel-timing > $O/c4_pmc_$pmc.log 2>&1
done
echo done

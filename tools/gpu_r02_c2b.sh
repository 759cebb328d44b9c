#!/bin/bash
# C2 K-split A/B: 512 vs 256 vs none
set -o pipefail
mkdir -p gpurun_out/r02c2c
for ks in 512; do
timeout -k 10 200 python bench.py --config C2 --steps 20 --warmup 3 --cpu-frames 0 --wn-opt ksplit=$ks > gpurun_out/r02c2c/bench_c2_ks$ks.json 2>> gpurun_out/r02c2c/err.log || exit 1
timeout -k 10 200 python bench.py --config C2 --no-graph --steps 10 --warmup 3 --cpu-frames 0 --wn-opt ksplit=$ks > gpurun_out/r02c2c/bench_c2e_ks$ks.json 2>> gpurun_out/r02c2c/err.log || exit 1
done

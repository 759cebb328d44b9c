#!/bin/bash
# r04 baseline counters: LVC phase split (s_memtime probe) + SQ passes for the top C3 and C5
# kernels.  usage (GPU box): tools/gpu_r04_base.sh <tag>
set -e
TAG=$1; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 120 tools/bin/lvc_probe 256 384 1 > $O/lvc_probe_final.txt 2>&1
timeout -k 10 400 tools/pmc_sq.sh $TAG/c3 "lvc_block_bf16|kp_kernel_bf16|wn_layer_bf16|dblock_bf16|kp_hidden_bf16" --steps 2
timeout -k 10 400 tools/pmc_sq.sh $TAG/c5 "nsf_|enc_|wn_layer_bf16" --config C5 --steps 1
python tools/pmc_sq.py $O/c3 > $O/c3_sq.txt
python tools/pmc_sq.py $O/c5 > $O/c5_sq.txt
echo done

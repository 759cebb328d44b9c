#!/bin/bash
# SQ-counter passes (one rocprofv3 run each) over a short bench for the kernels matching
# a regex; summarise with tools/pmc_sq.py.
# usage (GPU box): tools/pmc_sq.sh <tag> <regex> [bench args...]   e.g. --config C5 --steps 1
set -e
TAG=$1; RE=$2; shift 2
ARGS="$*"
[ -z "$ARGS" ] && ARGS="--steps 2"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "$RE" -d $O/sq$i -o run --output-format csv -- \
    python -u $R/bench.py $ARGS --warmup 1 --cpu-frames 0 --no-kernel-timing > $O/sq$i.log 2>&1
done
echo done

#!/bin/bash
# SQ-counter passes over a short C3 bench with extra bench.py args, for kernels matching a regex.
# usage (GPU box): tools/pmc_sq_cmd2.sh <tag> <regex> [bench args...]; summary via tools/pmc_sq.py
set -e
TAG=$1; RE=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-include-regex "$RE" -d $O/sq$i -o run --output-format csv -- \
    python -u $R/bench.py --steps 2 --warmup 1 --cpu-frames 0 --no-kernel-timing "$@" > $O/sq$i.log 2>&1
done
python $R/tools/pmc_sq.py $O > $O/summary.txt
cat $O/summary.txt

#!/bin/bash
# SQ-counter passes (one rocprofv3 run each) over a standalone probe binary.
# usage (GPU box): tools/pmc_sq_probe.sh <tag> <binary> [args...]; summary via tools/pmc_sq.py
set -e
TAG=$1; BIN=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA" \
           "SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $pmc -d $O/sq$i -o run --output-format csv -- $R/$BIN "$@" > $O/sq$i.log 2>&1
done
python $R/tools/pmc_sq.py $O > $O/summary.txt
cat $O/summary.txt

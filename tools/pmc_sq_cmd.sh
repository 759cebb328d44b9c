#!/bin/bash
# SQ/TA/TCP counter passes (one rocprofv3 run each) over an arbitrary python command for the kernels
# matching a regex; summarise with tools/pmc_sq.py.  usage (GPU box): tools/pmc_sq_cmd.sh <tag> <regex> <script> [args...]
set -e
TAG=$1; RE=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_max TA_TA_BUSY_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $pmc --kernel-include-regex "$RE" -d $O/sq$i -o run --output-format csv -- \
    python3 -u "$@" > $O/sq$i.log 2>&1
done
echo done

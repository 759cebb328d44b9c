#!/bin/bash
# Kernel-trace stats + separate PMC passes for one kernel of the FastDiff sampler.
# usage (on the GPU box): tools/prof_lvc.sh <tag> <kernel-regex>
# Env (e.g. PRODIFF_LVC_TS) is inherited by the profiled python process.
set -e
TAG=$1; RE=$2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
P="python $GRAFT_REPO_ROOT/tools/prof_fastdiff.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $P > $OUT.trace.log 2>&1
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --kernel-include-regex "$RE" -d $OUT/pmc$i -o run --output-format csv -- $P > $OUT.pmc$i.log 2>&1
done
echo done

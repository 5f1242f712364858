#!/bin/bash
# PMC passes (one counter group per rocprofv3 run; no tracing domains mixed in).
# usage: tools/pmc.sh <outdir-name> <kernel-regex>
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
RX=$2
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  SFM_AMD_LIB=${SFM_AMD_LIB:-} timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d $OUT/p$i -- python3 $R/tools/pmc_c3.py > $OUT.p$i.log 2>&1
done
echo done

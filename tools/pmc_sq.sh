#!/bin/bash
# SQ instruction / stall counters of the C3 solve's kernels (two passes of
# <= 8 SQ counters, no tracing), then per-kernel means (tools/pmcsum.py).
# usage: tools/pmc_sq.sh <outdir-name> <kernel-regex>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$2" --output-format csv -d $OUT/p$i -- python3 $R/tools/pmc_c3.py solve > $OUT/p$i.log 2>&1 || exit 1
done
python3 $R/tools/pmcsum.py $OUT

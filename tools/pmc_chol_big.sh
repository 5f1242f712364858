#!/bin/bash
# HBM traffic and MFMA-busy of the dense factor at n = 12000 (C4's reduced
# camera system): FETCH_SIZE, WRITE_SIZE, MFMA busy + GRBM in separate passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_chol_big
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "k_chol_fused" --output-format csv -d $OUT/p$i -- python3 $R/tools/chol_bench.py 12000 > $OUT/p$i.log 2>&1 || exit 1
done
python3 $R/tools/pmcsum.py $OUT

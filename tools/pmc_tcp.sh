#!/bin/bash
# L1 (TCP) -> L2 request counts of the Schur variants (env settings as args).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  tag=$(echo $v | tr '=' '_')
  for grp in "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"; do
    g=$(echo $grp | cut -c1-20 | tr ' ' '_')
    env $v timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_schur" --output-format csv -d $R/gpurun_out/pmct_$tag/$g -- python3 $R/tools/pmc_c3.py > $R/gpurun_out/pmct_$tag.$g.log 2>&1 || { echo "pmc failed $v $grp"; tail -3 $R/gpurun_out/pmct_$tag.$g.log; exit 1; }
  done
  echo "== $v"; python3 $R/tools/pmcsum.py $R/gpurun_out/pmct_$tag | grep -v schur_diag -A0
done

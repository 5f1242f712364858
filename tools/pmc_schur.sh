#!/bin/bash
# FETCH_SIZE / TCC hit-miss of k_schur under the env variants given as args (e.g. "SFM_SCHUR_XCD=1").
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  tag=$(echo $v | tr '=' '_')
  for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    g=$(echo $grp | tr ' ' '_')
    env $v timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_schur_row|k_schur$|k_schur\\(" --output-format csv -d $R/gpurun_out/pmcs_$tag/$g -- python3 $R/tools/pmc_c3.py > $R/gpurun_out/pmcs_$tag.$g.log 2>&1 || exit 1
  done
  echo "== $v"; python3 $R/tools/pmcsum.py $R/gpurun_out/pmcs_$tag
done

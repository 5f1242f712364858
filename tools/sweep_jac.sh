#!/bin/bash
# usage: tools/sweep_jac.sh v1 v2 ... — k_jacobian time (C3) per persistent-grid size
# (SFM_JAC_WG_PER_XCD workgroups per XCD slice)
set -o pipefail
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  echo -n "wg_per_xcd=$v "; SFM_JAC_WG_PER_XCD=$v timeout -k 10 120 python3 $R/tools/pmc_c3.py 2>&1 | grep jacobian || exit 1
done

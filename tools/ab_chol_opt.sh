#!/bin/bash
# A/B of the fused Cholesky's hand-off forms (SFM_CHOL_OPT bits) on one box:
# walker phase stamps (abvar/var_stamps.so) and the production factor time.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
for rep in 1 2; do
  for o in "$@"; do
    SFM_CHOL_OPT=$o timeout -k 10 60 python3 tools/walker_phases.py 3000 || exit 1
    SFM_CHOL_OPT=$o timeout -k 10 60 python3 tools/chol_scale.py 3000 6000 || exit 1
  done
done

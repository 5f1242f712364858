#!/bin/bash
# A/B of library builds abvar/var_<name>.so (and "cur" = sfm_amd/libsfm_amd.so)
# on one box: dense factor + solve at n = 3000 / 6000, alternating twice.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = cur ]; then unset SFM_AMD_LIB; else export SFM_AMD_LIB=$R/abvar/var_$v.so; fi
    echo "== $v"
    timeout -k 10 60 python3 tools/chol_scale.py 3000 6000 || exit 1
  done
done

#!/bin/bash
# k_jacobian (C3): warm (back to back) and cold (behind a 288-MB read of
# another buffer) per ablation build tools/var_<name>.so
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  echo -n "$v warm "; SFM_AMD_LIB=$R/tools/var_$v.so timeout -k 10 120 python3 $R/tools/pmc_c3.py 2>&1 | grep jacobian || exit 1
  echo -n "$v cold "; SFM_JAC_THRASH=2 SFM_AMD_LIB=$R/tools/var_$v.so timeout -k 10 120 python3 $R/tools/pmc_c3.py 2>&1 | grep jacobian || exit 1
done

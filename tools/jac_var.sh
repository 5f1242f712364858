#!/bin/bash
# Time k_jacobian in ablation builds tools/var_<name>.so (bench_jacobian, C3).
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  echo -n "$v "; SFM_AMD_LIB=$R/tools/var_$v.so timeout -k 10 120 python3 $R/tools/pmc_c3.py 2>&1 | grep jacobian
done

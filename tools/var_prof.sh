#!/bin/bash
# Profile ablation builds tools/var_*.so with tools/chol_bench.py (rocprofv3 kernel stats).
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  SFM_AMD_LIB=$R/tools/var_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/var_$v -- python3 $R/tools/chol_bench.py 3000 > $R/gpurun_out/var_$v.log 2>&1
  python3 $R/tools/kstats.py $R/gpurun_out/var_$v | grep -E "potrf|trsm|syrk|backsolve" | sed "s/^/$v /"
done

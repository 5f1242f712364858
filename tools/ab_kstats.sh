#!/bin/bash
# A/B kernel stats of tools/ab_solve.py under builds abvar/var_<name>.so, each
# variant twice in alternation (same box).
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for pass in 1 2; do
for v in "$@"; do
  rm -rf $R/gpurun_out/ab_${v}_$pass
  SFM_AMD_LIB=$R/abvar/var_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_${v}_$pass -- python3 $R/tools/ab_solve.py > $R/gpurun_out/ab_${v}_$pass.log 2>&1 || { echo "$v failed"; tail $R/gpurun_out/ab_${v}_$pass.log; exit 1; }
  grep final_cost $R/gpurun_out/ab_${v}_$pass.log | sed "s/^/$v /"
  python3 $R/tools/kstats.py $R/gpurun_out/ab_${v}_$pass | head -8 | sed "s/^/$v /"
done
done

#!/bin/bash
# rocprof kernel stats of tools/pmc_c3.py under ablation builds tools/var_<name>.so
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  rm -rf $R/gpurun_out/vk_$v
  SFM_AMD_LIB=$R/tools/var_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/vk_$v -- python3 $R/tools/pmc_c3.py > $R/gpurun_out/vk_$v.log 2>&1
  python3 $R/tools/kstats.py $R/gpurun_out/vk_$v | head -16 | sed "s/^/$v /"
done

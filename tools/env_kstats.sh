#!/bin/bash
# rocprof kernel stats of tools/pmc_c3.py (one solve) under env settings given
# as args, e.g. tools/env_kstats.sh SFM_SCHUR_PTS_SUB=8 SFM_SCHUR_PTS_SUB=16
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  tag=$(echo $v | tr '=' '_')
  rm -rf $R/gpurun_out/ek_$tag
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ek_$tag -- python3 $R/tools/pmc_c3.py solve > $R/gpurun_out/ek_$tag.log 2>&1 || exit 1
  python3 $R/tools/kstats.py $R/gpurun_out/ek_$tag | head -12 | sed "s/^/$v /"
done

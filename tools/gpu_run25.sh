#!/bin/bash
# C1 one-shot kernel mix (rocprofv3 kernel trace of tools/c1_latency.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r25
rm -rf $O && mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/tools/c1_latency.py > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
cat $O/c1.log
python3 $R/tools/kstats.py $O/prof

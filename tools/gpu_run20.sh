#!/bin/bash
# k_pnp_epnp kernel time (kernel trace of the bench pnp leg).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04j
rm -rf $O && mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/tools/leg.py pnp > $O/pnp.json 2> $O/pnp.err || exit 1
python3 $R/tools/kstats.py $O/prof > $O/kernel_stats_pnp.txt

#!/bin/bash
# PnP subsets cached per (n, iterations): PnP tests, the pnp leg and its trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04k
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_compat.py -x -q --timeout 200 --timeout-method thread > $O/pnp_tests.log 2>&1 || { tail -30 $O/pnp_tests.log; exit 1; }
timeout -k 10 120 python3 tools/leg.py pnp > $O/pnp.json 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/tools/leg.py pnp > /dev/null 2> $O/pnp.err || exit 1
python3 $R/tools/kstats.py $O/prof > $O/kernel_stats_pnp.txt

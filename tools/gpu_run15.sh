#!/bin/bash
# Small-problem setup sorts (one-launch radix sorts): GPU suite, C1 latency + timeline.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04e
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/c1_latency.py > $O/c1.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -- python3 $R/tools/c1_latency.py > $O/run.txt 2>&1 || exit 1
python3 $R/tools/c1_latency.py --summarise $O/trace > $O/summary.txt 2>&1

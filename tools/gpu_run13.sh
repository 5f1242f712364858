#!/bin/bash
# C1 one-shot timeline (kernel + memory-copy trace) and its summary.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c1tl
rm -rf $O && mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -- python3 $R/tools/c1_latency.py > $O/run.txt 2>&1 || exit 1
python3 $R/tools/c1_latency.py --summarise $O/trace > $O/summary.txt 2>&1

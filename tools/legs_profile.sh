#!/bin/bash
# Kernel-trace statistics of every bench leg, and the C1 keyframe one-shot
# timeline (tools/c1_latency.py --summarise), into gpurun_out/$TAG.
set -o pipefail
TAG=${1:-rxx}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
rm -rf $O && mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_all -- python3 $R/bench.py --no-cpu-baseline > $O/prof_all_bench.json 2> $O/prof_all_bench.err || exit 1
python3 $R/tools/kstats.py $O/prof_all > $O/kernel_stats_all_legs.txt || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/c1trace -- python3 $R/tools/c1_latency.py > $O/c1_run.txt 2>&1 || exit 1
python3 $R/tools/c1_latency.py --summarise $O/c1trace > $O/c1_summary.txt 2>&1

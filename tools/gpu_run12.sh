#!/bin/bash
# Round-4 batch 12: GPU suite, kernel trace of the C3 bench, bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04c
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-tracker --no-oneshot --steps 10 > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --no-cpu-baseline --no-tracker --no-oneshot > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
python3 $R/tools/kstats.py $O/prof > $O/kernel_stats_c3.txt

#!/bin/bash
# Round-4 batch 11: GPU suite, kernel trace of the C3 bench (observation-pass
# grid fix), the obs_prep / backsub traffic pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04b
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --no-cpu-baseline --no-tracker --no-oneshot > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
python3 $R/tools/kstats.py $O/prof > $O/kernel_stats_c3.txt || exit 1
timeout -k 10 900 bash $R/tools/pmc_traffic.sh > $O/pmc_traffic.txt 2>&1 || exit 1
python3 $R/tools/pmc_json.py $R/gpurun_out/pmc_traffic $O/pmc_c3.json > $O/pmc_json.txt 2>&1

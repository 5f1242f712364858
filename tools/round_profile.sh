#!/bin/bash
# Round-end measurement on one MI355X (gpurun): the default bench line, the
# kernel-trace statistics of the same bench command, then the PMC traffic
# passes (tools/pmc_traffic.sh).  Everything lands in gpurun_out/$TAG.
#   bash tools/round_profile.sh r03
set -o pipefail
TAG=${1:-rxx}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
# the C3 line alone (its kernels' averages are the roofline's), then every leg
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --no-cpu-baseline --no-tracker --no-oneshot > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
python3 $R/tools/kstats.py $O/prof > $O/kernel_stats_c3.txt || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_all -- python3 $R/bench.py --no-cpu-baseline > $O/prof_all_bench.json 2> $O/prof_all_bench.err || exit 1
python3 $R/tools/kstats.py $O/prof_all > $O/kernel_stats_all_legs.txt || exit 1
timeout -k 10 900 bash $R/tools/pmc_traffic.sh > $O/pmc_traffic.txt 2>&1 || exit 1

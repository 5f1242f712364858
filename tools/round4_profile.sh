#!/bin/bash
# Round-4 measurement on one MI355X (gpurun): the default bench line, the
# kernel-trace statistics of the C3 bench command (the roofline's kernels),
# the PMC traffic passes and the MFMA-busy pass (tools/pmc_traffic.sh,
# tools/pmc_mfma.sh).  Everything lands in gpurun_out/r04.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --no-cpu-baseline --no-tracker --no-oneshot > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
python3 $R/tools/kstats.py $O/prof > $O/kernel_stats_c3.txt || exit 1
timeout -k 10 900 bash $R/tools/pmc_traffic.sh > $O/pmc_traffic.txt 2>&1 || exit 1
python3 $R/tools/pmc_json.py $R/gpurun_out/pmc_traffic $O/pmc_c3.json > $O/pmc_json.txt 2>&1 || exit 1
timeout -k 10 200 bash $R/tools/pmc_mfma.sh > $O/pmc_mfma.txt 2>&1 || exit 1
cp $R/gpurun_out/pmc_mfma/pmc_mfma.json $O/pmc_mfma_c3.json
timeout -k 10 200 bash $R/tools/pmc_stall.sh > $O/pmc_stall.txt 2>&1 || exit 1
cp $R/gpurun_out/pmc_stall/pmc_stall.json $O/pmc_stall_c3.json

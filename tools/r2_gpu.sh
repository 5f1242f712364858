#!/bin/bash
# Round GPU pass: parity tests, bench line, rocprofv3 kernel stats of the bench.
# TAG names the outputs (gpurun_out/<TAG>_*).
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-r2}
cd $R
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/${T}_gpu_tests.log
fi
timeout -k 10 400 python -u bench.py --phases > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof_bench -- python3 $R/bench.py --no-cpu-baseline --no-tracker --no-oneshot > $R/gpurun_out/${T}_prof_bench.log 2>&1 || { echo "rocprof failed"; tail -20 $R/gpurun_out/${T}_prof_bench.log; exit 1; }
python3 $R/tools/kstats.py $R/gpurun_out/${T}_prof_bench

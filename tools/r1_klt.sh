#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_klt.py -x -v --timeout 120 --timeout-method thread > gpurun_out/klt_tests.log 2>&1 || { echo "klt tests failed"; tail -40 gpurun_out/klt_tests.log; exit 1; }
tail -3 gpurun_out/klt_tests.log
timeout -k 10 120 python -u tools/klt_bench.py 500 50 2>&1 | tee gpurun_out/klt_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_klt -- python3 $R/tools/klt_bench.py 500 50 > $R/gpurun_out/prof_klt.log 2>&1 || { echo "rocprof failed"; tail -20 $R/gpurun_out/prof_klt.log; exit 1; }
python3 $R/tools/kstats.py $R/gpurun_out/prof_klt

#!/bin/bash
# Onesweep setup sorts: C1 A/B, then the 3-rank sharded one-GPU test with the
# workers' stderr visible (-s).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r27
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 300 bash tools/ab_c1.sh onesweep= merge=:SFM_SORT_MERGE=1 > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
cat $O/c1.log
timeout -k 10 170 python -u -m pytest "tests/test_gpu_shards.py::test_sharded_solve_on_one_gpu_matches_single" -m gpu -x -v -s --timeout 150 --timeout-method thread > $O/shards.log 2>&1
rc=$?
tail -60 $O/shards.log
exit $rc

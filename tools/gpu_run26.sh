#!/bin/bash
# Onesweep setup sorts: whole GPU suite, then C1 one-shot and C3 setup with
# the onesweep sorts and with rocprim's default (merge sort below 2^20).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r26
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 bash tools/ab_c1.sh onesweep= merge=:SFM_SORT_MERGE=1 > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
cat $O/c1.log
for v in 0 1 0 1; do
  SFM_SORT_MERGE=$v timeout -k 10 200 python3 tools/c3_setup_timing.py 2>&1 | sed "s/^/merge=$v /" || exit 1
done

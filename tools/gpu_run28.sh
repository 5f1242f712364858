#!/bin/bash
# Whole GPU suite (-v: each test named as it starts) after the sort revert.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r28
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log

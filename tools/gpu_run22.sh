#!/bin/bash
# Round-end refresh: the default bench line and the whole GPU suite + smoke.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final2
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 500 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1

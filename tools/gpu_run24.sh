#!/bin/bash
# AcceptFold check: LM-branch parity (device loop vs host loop, bitwise),
# the parity suite, then the C1 one-shot latency with and without the fold.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r24
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_lm_branches.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 bash tools/ab_c1.sh fold= nofold=:SFM_NO_ACCEPT_FOLD=1 > $O/c1.log 2>&1 || { tail -20 $O/c1.log; exit 1; }
cat $O/c1.log

#!/bin/bash
# Jacobian padding-lane change: A/B against HEAD on the C3 bench, then the
# GPU tests that compare traces (LM branches, scale).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04f
rm -rf $O && mkdir -p $O
cd $R
bash tools/ab_bench.sh head cur > $O/ab_bench.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_lm_branches.py tests/test_gpu_scale.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for hp in 0 127 63 31; do
  echo "== helpers $hp" >> $O/helpers.txt
  SFM_CHOL_HELPERS=$hp timeout -k 10 60 python3 tools/chol_scale.py 3000 6000 >> $O/helpers.txt 2>&1 || exit 1
done

#!/bin/bash
# Row-parallel Jacobi sweep in the PnP SVD: the PnP GPU tests (bit-exact vs
# the oracle), the compat drop-in, then the pnp leg A/B against HEAD, stamps.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04i
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_pnp.py tests/test_gpu_compat.py tests/test_gpu_live.py -x -q --timeout 200 --timeout-method thread > $O/pnp_tests.log 2>&1 || { tail -30 $O/pnp_tests.log; exit 1; }
bash tools/ab_pnp.sh prev cur > $O/ab_pnp.txt 2>&1

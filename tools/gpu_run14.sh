#!/bin/bash
# Small-system Cholesky (one workgroup, nblk <= 2): the GPU suite, C1 latency.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04d
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python tools/c1_latency.py > $O/c1.txt 2>&1

#!/bin/bash
# Host-side set_problem checks for small problems: the GPU suite, C1 latency.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04l
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
timeout -k 10 120 python tools/c1_latency.py > $O/c1.txt 2>&1

#!/bin/bash
# Round-4 batch 8: Cholesky A/B (round-3 walker vs the restored walker with
# start-order roles), the full GPU suite + C3 bench, the emulated-rank
# validation against the pre-fix collectives.
set -o pipefail
mkdir -p gpurun_out
bash tools/ab_libs.sh r3 cur > gpurun_out/ab_libs.txt 2>&1 && \
bash tools/gpu_check.sh && \
bash tools/ab_bench.sh r3 cur > gpurun_out/ab_bench.txt 2>&1 && \
{ SFM_AMD_LIB=$GRAFT_REPO_ROOT/tools/var_nogate.so timeout -k 10 200 python -u -m pytest tests/test_gpu_lm_branches.py -k emulated -q --timeout 120 --timeout-method thread > gpurun_out/nogate.log 2>&1; echo "nogate rc=$? (the emulated two-rank test must FAIL on the pre-fix collectives)" >> gpurun_out/nogate.log; }

#!/bin/bash
# Round-4 batch 9: GPU suite + C3 bench, bench A/B against the round-3
# library, emulated-rank validation, the C4 single-GPU line, then the
# round-4 profiling passes (tools/round4_profile.sh).
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_check.sh && \
bash tools/ab_bench.sh r3 cur > gpurun_out/ab_bench.txt 2>&1 && \
{ SFM_AMD_LIB=$GRAFT_REPO_ROOT/tools/var_nogate.so timeout -k 10 200 python -u -m pytest tests/test_gpu_lm_branches.py -k emulated -q --timeout 120 --timeout-method thread > gpurun_out/nogate.log 2>&1; echo "nogate rc=$? (the emulated two-rank test must FAIL on the pre-fix collectives)" >> gpurun_out/nogate.log; } && \
timeout -k 10 400 python -u bench.py --gpus 1 --cams 2000 --total-pts 1000000 --no-tracker --no-oneshot > gpurun_out/c4_n1.json 2> gpurun_out/c4_n1.err && \
bash tools/round4_profile.sh

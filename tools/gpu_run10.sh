#!/bin/bash
# Round-4 batch 10: the C4 single-GPU line, then the round-4 profiling passes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gpus 1 --cams 2000 --total-pts 1000000 --no-tracker --no-oneshot --no-cpu-baseline > gpurun_out/c4_n1.json 2> gpurun_out/c4_n1.err && \
bash tools/round4_profile.sh

#!/bin/bash
# GPU check used during development: full GPU suite, dense factor across
# sizes, C3 bench without the tracker legs (writes gpurun_out/).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/chol_scale.py > gpurun_out/chol_scale.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-tracker --no-cpu-baseline --no-oneshot > gpurun_out/bench.json 2> gpurun_out/bench.err

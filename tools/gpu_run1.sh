set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-tracker --no-cpu-baseline --no-oneshot > gpurun_out/bench.json 2> gpurun_out/bench.err

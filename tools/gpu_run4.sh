set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 python tools/gauge_gpu.py > gpurun_out/gauge_gpu.txt 2>&1 && bash tools/ab_chol_opt.sh 0 1 2 4 7 > gpurun_out/ab_opt.txt 2>&1 && timeout -k 10 400 python -u -m pytest tests/test_gpu_concurrency.py -x -v --timeout 300 --timeout-method thread > gpurun_out/conc.log 2>&1 && bash tools/gpu_check.sh

set -o pipefail
mkdir -p gpurun_out
bash tools/ab_libs.sh r3 cur ext pub1 > gpurun_out/ab_libs.txt 2>&1 && \
timeout -k 10 60 python3 tools/walker_phases.py 3000 > gpurun_out/stamps.txt 2>&1 && \
SFM_AMD_LIB=$GRAFT_REPO_ROOT/tools/var_extst.so timeout -k 10 60 python3 tools/walker_phases.py 3000 >> gpurun_out/stamps.txt 2>&1 && \
timeout -k 10 60 python tools/gauge_gpu.py > gpurun_out/gauge_gpu.txt 2>&1 && \
bash tools/ab_bench.sh cur ext jac2 > gpurun_out/ab_bench.txt 2>&1 && \
bash tools/ab_pnp.sh prev cur > gpurun_out/ab_pnp.txt 2>&1 && \
timeout -k 10 120 python tools/c1_latency.py > gpurun_out/c1.txt 2>&1 && \
SFM_LM_GRAPH=1 timeout -k 10 120 python tools/c1_latency.py >> gpurun_out/c1.txt 2>&1 && \
bash tools/gpu_check.sh && \
{ SFM_AMD_LIB=$GRAFT_REPO_ROOT/tools/var_nogate.so timeout -k 10 200 python -u -m pytest tests/test_gpu_lm_branches.py -k emulated -q --timeout 120 --timeout-method thread > gpurun_out/nogate.log 2>&1; echo "nogate rc=$? (the emulated two-rank test must FAIL on the pre-fix collectives)" >> gpurun_out/nogate.log; }

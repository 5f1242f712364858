set -o pipefail
mkdir -p gpurun_out
bash tools/ab_libs.sh r3 c1 cur > gpurun_out/ab_libs.txt 2>&1 && \
SFM_CHOL_OPT=0 timeout -k 10 60 python3 tools/walker_phases.py 3000 > gpurun_out/stamps.txt 2>&1 && \
SFM_CHOL_OPT=7 timeout -k 10 60 python3 tools/walker_phases.py 3000 >> gpurun_out/stamps.txt 2>&1

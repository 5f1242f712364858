#!/bin/bash
# Round-end GPU pass: parity tests, bench, rocprofv3 kernel stats, then the
# MFMA-busy and HBM-traffic PMC passes (each pass its own run).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r2f} bash tools/r2_gpu.sh || exit 1
bash tools/pmc_mfma.sh > gpurun_out/${TAG:-r2f}_pmc_mfma.txt 2>&1 || { echo "pmc mfma failed"; tail gpurun_out/${TAG:-r2f}_pmc_mfma.txt; exit 1; }
cat gpurun_out/${TAG:-r2f}_pmc_mfma.txt
bash tools/pmc_traffic.sh > gpurun_out/${TAG:-r2f}_pmc_traffic.txt 2>&1 || { echo "pmc traffic failed"; tail gpurun_out/${TAG:-r2f}_pmc_traffic.txt; exit 1; }
echo traffic ok

#!/bin/bash
# HBM traffic per launch (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes (no tracing mixed in), C3 workload (tools/pmc_c3.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
RX='k_jacobian|k_chol_fused|k_schur|k_obs_prep|k_backsolve|k_point_eval|k_cam_reduce|k_backsub'
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $OUT/fetch -- python3 $R/tools/pmc_c3.py > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $OUT/write -- python3 $R/tools/pmc_c3.py > $OUT/write.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$RX" --output-format csv -d $OUT/hit -- python3 $R/tools/pmc_c3.py > $OUT/hit.log 2>&1 || exit 1
python3 $R/tools/pmcsum.py $OUT

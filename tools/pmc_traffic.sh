#!/bin/bash
# HBM traffic per launch (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and WRITE_SIZE
# in separate --pmc passes (no tracing mixed in), C3 workload (tools/pmc_c3.py):
# k_jacobian on the record-writing passes, the production kernels on one
# solve; first the known-byte calibration kernels (tools/pmc_calib.hip).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_traffic
rm -rf $OUT && mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
RXS='k_chol_fused|k_schur|k_obs_prep|k_backsolve|k_point_eval|k_cam_sum|k_backsub|k_point_factor|k_jacobian'
for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_HIT_sum TCC_MISS_sum:hit"; do
  ctr=${pass%%:*}; name=${pass##*:}
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $OUT/${name}_calib -- $R/tools/pmc_calib > $OUT/${name}_calib.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex 'k_jacobian' --output-format csv -d $OUT/${name}_jac -- python3 $R/tools/pmc_c3.py jac > $OUT/${name}_jac.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$RXS" --output-format csv -d $OUT/${name}_solve -- python3 $R/tools/pmc_c3.py solve > $OUT/${name}_solve.log 2>&1 || exit 1
done
python3 $R/tools/pmcsum.py $OUT

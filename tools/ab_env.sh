#!/bin/bash
# A/B kernel stats of tools/ab_solve.py (C3 solve) under environment variants:
#   bash tools/ab_env.sh base='' j128='SFM_JAC_WG_PER_XCD=128' head='SFM_AMD_LIB=abvar/var_head.so' ...
# each variant twice in alternation (same box); prints the final cost and the
# top kernels of each run.  AB_CMD='tools/leg.py pnp' profiles another script.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for pass in 1 2; do
for spec in "$@"; do
  label=${spec%%=*}; vars=${spec#*=}
  rm -rf $R/gpurun_out/ab_${label}_$pass
  (
    for kv in $vars; do
      case $kv in SFM_AMD_LIB=*) export SFM_AMD_LIB=$R/${kv#SFM_AMD_LIB=} ;; *) export "$kv" ;; esac
    done
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_${label}_$pass -- python3 $R/${AB_CMD:-tools/ab_solve.py} > $R/gpurun_out/ab_${label}_$pass.log 2>&1
  ) || { echo "$label failed"; tail $R/gpurun_out/ab_${label}_$pass.log; exit 1; }
  grep -E "final_cost|ms_per_call|\"inliers" $R/gpurun_out/ab_${label}_$pass.log | sed "s/^/$label /"
  python3 $R/tools/kstats.py $R/gpurun_out/ab_${label}_$pass | grep -E "${KRX:-k_jacobian|k_obs_prep|k_cam_sum|k_schur_diag|k_chol|k_schur_pts}" | sed "s/^/$label /"
done
done

set -e
R=$GRAFT_REPO_ROOT
cd $R
cp sfm_amd/libsfm_amd.so tools/var_new.so
timeout -k 5 30 tools/panel_micro > gpurun_out/panel_micro.txt 2>&1
timeout -k 10 400 bash tools/ab_kstats.sh old new > gpurun_out/ab2.txt 2>&1
timeout -k 10 300 bash tools/pmc_ab.sh k_schur_pts old new > gpurun_out/pmc_ab2.txt 2>&1
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_lm_branches.py tests/test_gpu_parity.py tests/test_gpu_shards.py -k "not c4" > gpurun_out/r3_par2.log 2>&1

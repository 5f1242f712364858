#!/bin/bash
# Overlap variant 2 (full helper grid dispatched beside the Schur pass): C3
# parity subset with it on, then the C3 bench alternating 0 / 2, then the
# round-4 profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04h
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "small_system or dense_cholesky" --timeout 150 --timeout-method thread > $O/small_tests.log 2>&1 || { tail -30 $O/small_tests.log; exit 1; }
SFM_OVERLAP=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -q -k "baseline_sizes or reproducible or c4_single" --timeout 200 --timeout-method thread > $O/ov_tests.log 2>&1 || { tail -30 $O/ov_tests.log; exit 1; }
for rep in 1 2; do
  for ov in 0 2; do
    SFM_OVERLAP=$ov timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-tracker --no-oneshot --steps 10 2>>$O/bench.err | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('overlap=$ov', 'ms_per_step', round(d['ms_per_step'],3), d['phase_ms_per_solve'])" >> $O/ab.txt || exit 1
  done
done
bash tools/round4_profile.sh

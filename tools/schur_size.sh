#!/bin/bash
# Schur time per launch vs point count at 500 cameras (does the F table
# fitting the 256-MB Infinity Cache change the per-pair rate?)
R=$GRAFT_REPO_ROOT
cd $R
for p in 50000 100000 150000 200000 300000; do
  echo -n "pts=$p: "
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-tracker --steps 5 --pts-per-gpu $p 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); ph=d['phase_ms_per_solve']; n=d['jacobian_evals_per_solve']
print('schur/launch', round(ph['schur']/d['lm_iterations_per_solve'],4), 'ms  obs', d['config']['observations'], 'iters', d['lm_iterations_per_solve'])" || exit 1
done

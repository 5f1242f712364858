#!/bin/bash
# usage: tools/sweep_env.sh VAR v1 v2 ...  — bench phases per value of an env knob
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
VAR=$1; shift
for v in "$@"; do
  env $VAR=$v timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-tracker --steps 10 > gpurun_out/sweep_$v.json 2> gpurun_out/sweep_$v.err || { echo "failed at $v"; tail -5 gpurun_out/sweep_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/sweep_$v.json').read().strip().splitlines()[-1])
print('$VAR=$v', 'ms_per_step', round(d['ms_per_step'],3), 'cost', d['final_cost'], d['phase_ms_per_solve'])"
done

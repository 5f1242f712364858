#!/bin/bash
# C3 solve with and without the Schur / Cholesky overlap (SFM_OVERLAP=1), alternating twice.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
for rep in 1 2; do for ov in 0 1; do
  SFM_OVERLAP=$ov timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-tracker --steps 10 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ov=$ov', round(d['ms_per_step'],3), d['phase_ms_per_solve'])" || exit 1
done; done

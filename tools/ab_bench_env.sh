#!/bin/bash
# C3 bench line (ms per solve and phases) under environment variants, alternating twice:
#   bash tools/ab_bench_env.sh serial=SFM_EVAL_SERIAL=1 split=
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
for rep in 1 2; do
  for spec in "$@"; do
    label=${spec%%=*}; vars=${spec#*=}
    ( for kv in $vars; do export "$kv"; done
      timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-tracker --steps 10 2>/dev/null ) | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],3), d['phase_ms_per_solve'], d['oneshot']['ms_per_solve'] if 'oneshot' in d else '')" || exit 1
  done
done

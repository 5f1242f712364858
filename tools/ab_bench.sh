#!/bin/bash
# A/B of library builds (abvar/var_<name>.so, "cur" = the in-tree library) on
# the C3 bench line, alternating twice: ms per solve and the phase times.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = cur ]; then unset SFM_AMD_LIB; else export SFM_AMD_LIB=$R/abvar/var_$v.so; fi
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-tracker --no-oneshot --steps 10 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$v', 'ms_per_step', round(d['ms_per_step'],3), 'jac_ms', d['roofline_jacobian']['avg_launch_ms'], 'chol_ms', d['roofline_cholesky']['avg_ms'], d['phase_ms_per_solve'])" || exit 1
  done
done

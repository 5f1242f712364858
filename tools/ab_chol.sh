#!/bin/bash
# A/B of library builds abvar/var_<name>.so on one box: dense Cholesky at
# n = 3000 / 12000 and the C3 bench phases, alternating twice.
R=$GRAFT_REPO_ROOT
cd $R
for rep in 1 2; do
  for v in "$@"; do
    echo "== $v"
    SFM_AMD_LIB=$R/abvar/var_$v.so timeout -k 10 120 python3 tools/chol_scale.py 3000 12000 || exit 1
    SFM_AMD_LIB=$R/abvar/var_$v.so timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-tracker --steps 10 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ms_per_step', round(d['ms_per_step'],3), d['phase_ms_per_solve'])" || exit 1
  done
done

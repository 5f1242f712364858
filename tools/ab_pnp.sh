#!/bin/bash
# A/B of library builds on the per-frame PnP leg (bench pnp_leg), alternating twice.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = cur ]; then unset SFM_AMD_LIB; else export SFM_AMD_LIB=$R/abvar/var_$v.so; fi
    timeout -k 10 120 python3 tools/leg.py pnp | python3 -c "import json,sys; d=json.load(sys.stdin); print('$v', 'pnp ms_per_call', round(d['ms_per_call'],4), 'inliers', d['inliers'])" || exit 1
  done
done

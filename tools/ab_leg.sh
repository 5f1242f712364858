#!/bin/bash
# A/B of library builds on one bench leg (tools/leg.py), alternating twice:
#   bash tools/ab_leg.sh live_path v10 cur     (abvar/var_<name>.so; cur = sfm_amd/libsfm_amd.so)
# prints the leg's headline figure per run (ms_per_frame / ms_per_call / c_abi_ms_per_solve).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
leg=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = cur ]; then unset SFM_AMD_LIB; else export SFM_AMD_LIB=$R/abvar/var_$v.so; fi
    timeout -k 10 300 python3 tools/leg.py $leg > /tmp/ab_leg.json 2>/dev/null || { echo "$v failed"; exit 1; }
    python3 -c "
import json; d=json.load(open('/tmp/ab_leg.json'))
k=[x for x in ('ms_per_frame','ms_per_call','c_abi_ms_per_solve','ms_per_solve') if x in d]
print('$v', {x: round(d[x], 4) for x in k}, d.get('host_s', ''))"
  done
done

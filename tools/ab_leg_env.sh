#!/bin/bash
# A/B of environment settings on one bench leg (tools/leg.py), alternating twice:
#   bash tools/ab_leg_env.sh live_path fused= composed=SFM_LIVE_COMPOSED=1
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
leg=$1; shift
for rep in 1 2; do
  for spec in "$@"; do
    label=${spec%%=*}; vars=${spec#*=}
    ( for kv in $vars; do export "$kv"; done
      timeout -k 10 300 python3 tools/leg.py $leg > /tmp/ab_leg.json 2>/dev/null ) || { echo "$label failed"; exit 1; }
    python3 -c "
import json; d=json.load(open('/tmp/ab_leg.json'))
k=[x for x in ('ms_per_frame','ms_per_call','c_abi_ms_per_solve','ms_per_solve') if x in d]
print('$label', {x: round(d[x], 4) for x in k}, d.get('host_s', ''))"
  done
done

#!/bin/bash
# Schur split-path chunk size at C1 / C2 (resident solve phases), and C3 with the split path forced.
R=$GRAFT_REPO_ROOT
cd $R
for pp in 8 16 32 64; do
  for cfg in C1 C2; do
    echo -n "pairs=$pp $cfg: "; CFG=$cfg SFM_SCHUR_SPLIT_PAIRS=$pp timeout -k 10 120 python3 tools/c1_latency.py | tail -2 | tr '\n' ' '; echo
  done
done
for pp in 24 72; do
  echo -n "C3 split pairs=$pp: "; SFM_SCHUR_SPLIT_MAXBLK=1000000 SFM_SCHUR_SPLIT_PAIRS=$pp timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-tracker --steps 5 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3), d['phase_ms_per_solve']['schur'])"
done

#!/bin/bash
# Resident-solve phase times of the keyframe-sized configs under each Schur
# formulation: split (pair chunks), recomputed-F blocks at 64/32/16 lanes.
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in C1 C2; do
  for v in "SFM_SCHUR_SPLIT=1" "SFM_SCHUR_SPLIT=0 SFM_SCHUR_PTS_SUB=64" "SFM_SCHUR_SPLIT=0 SFM_SCHUR_PTS_SUB=32" "SFM_SCHUR_SPLIT=0 SFM_SCHUR_PTS_SUB=16"; do
    echo "== $cfg $v"
    env CFG=$cfg $v timeout -k 10 120 python -u tools/c1_latency.py 2>&1 | tail -2 || exit 1
  done
done

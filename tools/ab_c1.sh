#!/bin/bash
# A/B of the C1 keyframe-sized one-shot latency (tools/c1_latency.py) between
# library builds / environments on one box, alternating:
#   bash tools/ab_c1.sh head=abvar/var_head.so new= devsetup=:SFM_HOST_SETUP=0
# (label=LIB[:VAR=VALUE ...]; an empty LIB is the in-tree library)
R=$GRAFT_REPO_ROOT
for pass in $(seq 1 ${PASSES:-2}); do
for spec in "$@"; do
  label=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""
  [ "$rest" != "$lib" ] && envs=${rest#*:}
  (
    if [ -n "$lib" ]; then export SFM_AMD_LIB=$R/$lib; else unset SFM_AMD_LIB; fi
    for kv in ${envs//:/ }; do export "$kv"; done
    timeout -k 10 120 python3 $R/tools/c1_latency.py 2>&1 | sed "s/^/$label /"
  ) || exit 1
done
done

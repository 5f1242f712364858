#!/bin/bash
# Kernel-level A/B of the C1 solve: a rocprofv3 kernel + copy trace of
# tools/c1_latency.py per library, summarised (per-kernel time per solve and
# the last solve's timeline) into gpurun_out/c1tab/LABEL.txt.
#   bash tools/c1_trace_ab.sh head=abvar/var_head.so new=
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c1tab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  label=${spec%%=*}; lib=${spec#*=}
  if [ -n "$lib" ]; then export SFM_AMD_LIB=$R/$lib; else unset SFM_AMD_LIB; fi
  rm -rf $O/tr_$label
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_$label -- python3 $R/tools/c1_latency.py > $O/$label.run.txt 2>&1 || exit 1
  python3 $R/tools/c1_latency.py --summarise $O/tr_$label > $O/$label.txt || exit 1
  rm -rf $O/tr_$label
done

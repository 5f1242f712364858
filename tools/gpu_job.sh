#!/bin/bash
# One GPU job = a list of steps, each under its own time limit, stopped at the
# first failure (never retried).  Replaces the one-off gpu_runN.sh scripts.
#
#   tools/gpu_job.sh NAME  SECONDS 'command' [SECONDS 'command' ...]
#
# Step k writes gpurun_out/NAME/k.log; the tail of a failing step is printed,
# and the job ends there.  Shorthands for common steps:
#   tests          the whole -m gpu suite (-v, per-test timeout)
#   tests:EXPR     the -m gpu tests matching -k EXPR
#   bench          bench.py default line -> gpurun_out/NAME/bench.json
#   kstats         rocprofv3 kernel trace of the C3 bench -> gpurun_out/NAME/kt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
name=$1; shift
O=$R/gpurun_out/$name
rm -rf "$O" && mkdir -p "$O"
export TMPDIR=/tmp
k=0
while [ $# -ge 2 ]; do
  secs=$1; cmd=$2; shift 2
  k=$((k + 1))
  case "$cmd" in
    tests) cmd="python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" ;;
    tests:*) cmd="python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k '${cmd#tests:}'" ;;
    bench) cmd="python bench.py > $O/bench.json" ;;
    kstats) cmd="rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 --no-tracker --no-cpu-baseline --no-oneshot --no-stream-copy > $O/kt_bench.json" ;;
  esac
  echo "== step $k (${secs}s): $cmd" | tee -a "$O/steps.txt"
  start=$(date +%s.%N)
  timeout -k 10 "$secs" bash -c "$cmd" > "$O/$k.log" 2>&1
  rc=$?
  end=$(date +%s.%N)
  echo "   rc=$rc  $(awk "BEGIN{printf \"%.1f\", $end - $start}") s" | tee -a "$O/steps.txt"
  if [ $rc -ne 0 ]; then
    tail -40 "$O/$k.log"
    exit $rc
  fi
  tail -5 "$O/$k.log"
done

#!/bin/bash
# GPU test pass: the given test paths (default: all) under -m gpu, one process,
# per-test timeout; log under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LOG=gpurun_out/${LOG_NAME:-gpu_tests}.log
timeout -k 10 ${TOTAL_TIMEOUT:-900} python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 120 --timeout-method thread -rs > $LOG 2>&1
rc=$?
tail -25 $LOG
exit $rc

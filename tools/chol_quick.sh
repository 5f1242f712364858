#!/bin/bash
# Cholesky iteration: dense-solve parity tests, factor timing across sizes,
# C3 solve parity + bench without the CPU/tracker legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-cq}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 200 python -u tools/chol_scale.py 3000 6000 12000 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-tracker --no-oneshot > gpurun_out/${T}_bench.json 2>/dev/null || { echo "bench failed"; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${T}_bench.json'));print('ms/solve',d['ms_per_step'],'chol',d['roofline']['avg_ms'],d['phase_ms_per_solve'])"

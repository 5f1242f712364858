#!/bin/bash
# Quick GPU check of a BA-kernel change: dense Cholesky across sizes, the BA
# parity tests, and the C3 bench line without the CPU / tracker legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-quick}
timeout -k 10 120 python -u tools/chol_scale.py 3000 6000 12000 > gpurun_out/${T}_chol.log 2>&1 || { echo "chol failed"; cat gpurun_out/${T}_chol.log; exit 1; }
cat gpurun_out/${T}_chol.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_lm_branches.py tests/test_gpu_shards.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-tracker --no-oneshot --steps 10 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print('ms/solve', round(d['ms_per_step'],3), 'chol', d['roofline_cholesky']['avg_ms'], 'frac', d['roofline_cholesky']['frac'], d['phase_ms_per_solve'])"

set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03b
rm -rf $O && mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $R/bench.py --no-cpu-baseline --no-tracker --no-oneshot > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
python3 $R/tools/kstats.py $O/prof > $O/kernel_stats_c3.txt

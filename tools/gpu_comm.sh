set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -v --timeout 120 --timeout-method thread -k "one_rank" > gpurun_out/t_comm.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_comm.log; exit 1; }
tail -5 gpurun_out/t_comm.log
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 --comm --no-cpu-baseline --no-tracker > gpurun_out/bench_comm.json 2> gpurun_out/bench_comm.err || { echo "bench failed"; tail -20 gpurun_out/bench_comm.err; exit 1; }
cat gpurun_out/bench_comm.json

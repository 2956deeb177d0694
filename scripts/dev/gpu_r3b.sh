# round-3 GPU session B: kernel tests for the changed kernels, batched FedAvg,
# headline bench, then kernel traces
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv.py tests/test_sketch_plan.py tests/test_fedavg_batched.py -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/r3_pytest_b.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3_pytest_b.log; exit 1; }
tail -2 gpurun_out/r3_pytest_b.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r3_bench_b.log 2>&1
tail -1 gpurun_out/r3_bench_b.log | cut -c1-200
for fb in on off; do
  timeout -k 10 400 python -u scripts/bench_configs.py --config cifar100_fedavg_local --steps 3 --warmup 1 -- --fedavg_batched $fb > gpurun_out/r3_fedavg_local_$fb.log 2>&1 || echo "bench $fb rc=$?"
  tail -1 gpurun_out/r3_fedavg_local_$fb.log
done
bash scripts/dev/prof_r3.sh

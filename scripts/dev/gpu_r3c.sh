# round-3 GPU session C: attention rework tests + GPT-2 config, batched FedAvg bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_transformer.py tests/test_fedavg_batched.py -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/r3_pytest_c.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3_pytest_c.log; exit 1; }
tail -2 gpurun_out/r3_pytest_c.log
timeout -k 10 300 python -u scripts/bench_configs.py --config gpt2_sketch > gpurun_out/r3_gpt2_c.log 2>&1
tail -1 gpurun_out/r3_gpt2_c.log
timeout -k 10 400 python -u scripts/bench_configs.py --config cifar100_fedavg_local --steps 3 --warmup 1 -- --fedavg_batched on > gpurun_out/r3_fedavg_local_on.log 2>&1 || echo "fedavg bench rc=$?"
tail -2 gpurun_out/r3_fedavg_local_on.log
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gpt2c -o tr -- python3 scripts/bench_configs.py --config gpt2_sketch --steps 4 --warmup 2 > gpurun_out/prof_gpt2c.log 2>&1
python3 scripts/round_kernels.py $(find gpurun_out/prof_gpt2c -name "*kernel_trace.csv" | head -1) --rounds 3 --top 40 > gpurun_out/r3_gpt2c_round_kernels.txt
head -25 gpurun_out/r3_gpt2c_round_kernels.txt

# secondary BASELINE configs, 1 GPU (logs under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/${1:-r3_secondary}.jsonl
: > $OUT
run() { timeout -k 10 ${1} python3 -u scripts/bench_configs.py "${@:2}" > gpurun_out/sec_tmp.log 2>&1 || { echo "FAIL $*"; tail -20 gpurun_out/sec_tmp.log; exit 1; }; tail -1 gpurun_out/sec_tmp.log | tee -a $OUT; }
run 300 --config imagenet_local_topk --steps 6 --warmup 2
run 300 --config cifar100_fedavg_local --steps 3 --warmup 1 -- --fedavg_batched on
run 300 --config cifar100_fedavg_local --steps 2 --warmup 1 -- --fedavg_batched off
run 300 --config cifar100_fedavg --steps 6 --warmup 2
run 300 --config gpt2_sketch --steps 6 --warmup 2

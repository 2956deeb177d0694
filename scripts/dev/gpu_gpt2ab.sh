# GPT-2 junction kernels: tests + round time
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpt2ab_tests.log 2>&1 || { tail -30 gpurun_out/gpt2ab_tests.log; exit 1; }
tail -1 gpurun_out/gpt2ab_tests.log
for i in 1 2; do timeout -k 10 300 python3 scripts/bench_configs.py --config gpt2_sketch --steps 10 --warmup 3 2>&1 | tail -1 | cut -c1-140 || exit 1; done

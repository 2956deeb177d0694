# GPT-2 round: native wgrad GEMM vs hipBLASLt, alternating on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 300 python3 scripts/bench_configs.py --config gpt2_sketch --steps 10 --warmup 3 2>&1 | tail -1 | cut -c1-120 || exit 1
  COMMEFF_WGRAD_GEMM=blas timeout -k 10 300 python3 scripts/bench_configs.py --config gpt2_sketch --steps 10 --warmup 3 2>&1 | tail -1 | cut -c1-120 || exit 1
done

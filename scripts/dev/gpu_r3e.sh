# attention hoist check + secondary configs + GPT-2 round profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer.py -x -q -m gpu -k attention --timeout 120 --timeout-method thread > gpurun_out/r3e_attn_tests.log 2>&1 || { tail -30 gpurun_out/r3e_attn_tests.log; exit 1; }
tail -1 gpurun_out/r3e_attn_tests.log
timeout -k 10 120 python3 scripts/bench_attention.py --p 0.1 || exit 1
bash scripts/dev/gpu_secondary.sh r3_secondary_b || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gpt2e -o tr -- python3 scripts/bench_configs.py --config gpt2_sketch --steps 4 --warmup 2 > gpurun_out/prof_gpt2e.log 2>&1 || exit 1
python3 scripts/round_kernels.py $(find gpurun_out/prof_gpt2e -name "*kernel_trace.csv" | head -1) --marker enc_p1 --rounds 3 --top 80 > gpurun_out/r3e_gpt2_round_kernels.txt 2>&1
head -3 gpurun_out/r3e_gpt2_round_kernels.txt
rm -rf gpurun_out/prof_gpt2e
echo ALLDONE

# kernel traces of the headline bench and the GPT-2 config (round-3 baseline)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_head -o tr -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_head.log 2>&1
python3 scripts/round_kernels.py gpurun_out/prof_head/*/tr_kernel_trace.csv --rounds 8 --top 60 > gpurun_out/r3_head_round_kernels.txt 2>&1 || python3 scripts/round_kernels.py $(find gpurun_out/prof_head -name "*kernel_trace.csv" | head -1) --rounds 8 --top 60 > gpurun_out/r3_head_round_kernels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gpt2 -o tr -- python3 scripts/bench_configs.py --config gpt2_sketch --steps 4 --warmup 2 > gpurun_out/prof_gpt2.log 2>&1
python3 scripts/round_kernels.py $(find gpurun_out/prof_gpt2 -name "*kernel_trace.csv" | head -1) --rounds 3 --top 70 > gpurun_out/r3_gpt2_round_kernels.txt
echo PROF_DONE

# GPT-2 round kernel trace, kept for the stream timeline
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_gpt2t -o tr -- python3 scripts/bench_configs.py --config gpt2_sketch --steps 4 --warmup 2 > gpurun_out/prof_gpt2t.log 2>&1
tail -1 gpurun_out/prof_gpt2t.log

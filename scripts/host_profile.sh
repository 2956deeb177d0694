#!/bin/bash
# Host-side (Python) profile of the round loop: cProfile over the 1-GPU bench
# (default) or a secondary config (CONFIG=gpt2_sketch), top functions by own
# time and by cumulative time -> gpurun_out/hp_stats.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$CONFIG" ]; then
  CMD="scripts/bench_configs.py --config $CONFIG --steps ${STEPS:-30} --warmup 3"
else
  CMD="bench.py --steps 600 --warmup 50"
fi
timeout -k 10 300 python -m cProfile -o gpurun_out/bench.prof $CMD > gpurun_out/hp_bench.log 2>&1 || exit $?
python -c "
import pstats; p=pstats.Stats('gpurun_out/bench.prof'); p.sort_stats('tottime').print_stats(60); p.sort_stats('cumtime').print_stats(90)" > gpurun_out/hp_stats.txt 2>&1
tail -1 gpurun_out/hp_bench.log

export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/bench.prof bench.py --steps 600 --warmup 50 > gpurun_out/hp_bench.log 2>&1 && python -c "
import pstats; p=pstats.Stats('gpurun_out/bench.prof'); p.sort_stats('tottime').print_stats(45); p.sort_stats('cumtime').print_stats(70)" > gpurun_out/hp_stats.txt 2>&1; tail -1 gpurun_out/hp_bench.log

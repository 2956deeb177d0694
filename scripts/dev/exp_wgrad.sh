#!/bin/bash
# halo wgrad: conv + grouped tests, bench 3 vs 2 stages, kernel trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv.py tests/test_grouped.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_test.log 2>&1 && \
COMMEFF_WGRAD_HALO_STAGES=2 timeout -k 10 300 python -u -m pytest tests/test_conv.py -x -q -k wgrad --timeout 120 --timeout-method thread > gpurun_out/conv_test2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_s3.log 2>&1 && \
COMMEFF_WGRAD_HALO_STAGES=2 timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_s2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_s3b.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/rocprof.log 2>&1
rc=$?
tail -n 3 gpurun_out/conv_test*.log gpurun_out/bench_*.log | cut -c1-300
exit $rc

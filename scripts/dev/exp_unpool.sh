#!/bin/bash
# fused unpool: its tests first, then the whole GPU suite, bench, trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv.py -x -q -k "unpool or kept_conv" --timeout 120 --timeout-method thread > gpurun_out/unpool_test.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_a.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_b.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/rocprof.log 2>&1
rc=$?
tail -n 3 gpurun_out/unpool_test.log gpurun_out/pytest_gpu.log gpurun_out/bench_*.log | cut -c1-250
exit $rc

#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv.py -x -q -k "unpool or kept_conv or residual or resnet9" --timeout 120 --timeout-method thread > gpurun_out/dual_test.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_a.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/rocprof.log 2>&1
rc=$?
tail -n 1 gpurun_out/dual_test.log gpurun_out/pytest_gpu.log; tail -n 1 gpurun_out/bench_a.log | cut -c100-190
exit $rc

#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops.py tests/test_sketch_plan.py tests/test_engine.py tests/test_graph.py tests/test_distributed.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/topk_test.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_a.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/rocprof.log 2>&1
rc=$?
tail -n 1 gpurun_out/topk_test.log; tail -n 1 gpurun_out/bench_a.log | cut -c100-190
exit $rc

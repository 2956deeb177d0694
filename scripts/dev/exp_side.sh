#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv.py -x -q -k "side_stream or kept_conv or unpool" --timeout 120 --timeout-method thread > gpurun_out/side_test.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_on1.log 2>&1 && \
COMMEFF_WGRAD_SIDE_REDUCE=0 timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_off1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_on2.log 2>&1 && \
COMMEFF_WGRAD_SIDE_REDUCE=0 timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_off2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/rocprof.log 2>&1
rc=$?
tail -n 1 gpurun_out/side_test.log; for f in gpurun_out/bench_o*.log; do echo $f; tail -n 1 $f | cut -c100-190; done
exit $rc

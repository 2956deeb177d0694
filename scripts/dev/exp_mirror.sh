#!/bin/bash
# kept weight copies: targeted tests, full GPU suite, headline bench, GPT-2 config
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv.py tests/test_transformer.py -x -q -k "kept_conv or replica or unpool" --timeout 120 --timeout-method thread > gpurun_out/mirror_test.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_a.log 2>&1 && \
timeout -k 10 400 python scripts/bench_configs.py --config gpt2_sketch > gpurun_out/gpt2.log 2>&1
rc=$?
tail -n 2 gpurun_out/mirror_test.log gpurun_out/pytest_gpu.log gpurun_out/bench_a.log gpurun_out/gpt2.log | cut -c1-250
exit $rc

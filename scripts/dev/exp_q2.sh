#!/bin/bash
# dense query Q2 with 16-byte run loads: sketch tests, GPT-2-size codec with / without
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sketch_plan.py tests/test_ops.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/sk_test.log 2>&1 && \
timeout -k 10 300 python scripts/bench_codec.py gpt2 > gpurun_out/codec_v4.log 2>&1 && \
COMMEFF_Q2_V4=0 timeout -k 10 300 python scripts/bench_codec.py gpt2 > gpurun_out/codec_nov4.log 2>&1
rc=$?
tail -n 2 gpurun_out/sk_test.log gpurun_out/codec_*.log | cut -c1-400
exit $rc

#!/bin/bash
# experiment: halo-64 conv tests, then exact vs dense sketch plan at ResNet-9 size
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv.py -x -q -k "halo_64 or dgrad or large_batch or unit_autograd" --timeout 120 --timeout-method thread > gpurun_out/conv_test.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_exact.log 2>&1 && \
COMMEFF_CONV_HALO64=0 timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_nohalo64.log 2>&1 && \
timeout -k 10 300 python scripts/bench_codec.py resnet9 > gpurun_out/codec_exact.log 2>&1 && \
COMMEFF_SKETCH_PLAN=dense timeout -k 10 300 python scripts/bench_codec.py resnet9 > gpurun_out/codec_dense.log 2>&1 && \
COMMEFF_SKETCH_PLAN=dense timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench_dense.log 2>&1
rc=$?
tail -n 3 gpurun_out/conv_test.log gpurun_out/codec_*.log gpurun_out/bench_*.log
exit $rc

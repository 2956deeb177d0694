# round-4 GPU check: benches first (kept even if a test fails), then tests
mkdir -p gpurun_out/r4e
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --round-times > gpurun_out/r4e/b20_5.log 2>&1 || { tail -20 gpurun_out/r4e/b20_5.log; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --warmup 50 > gpurun_out/r4e/b200_50.log 2>&1 || exit 1
COMMEFF_CONV_PIPE=0 timeout -k 10 300 python bench.py --steps 200 --warmup 50 > gpurun_out/r4e/b200_50_nopipe.log 2>&1 || exit 1
COMMEFF_TAPE=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --round-times > gpurun_out/r4e/b20_5_notape.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_conv.py > gpurun_out/r4e/conv.log 2>&1 || exit 1
COMMEFF_CONV_PIPE=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv.py -k "fwd or dgrad or pool or residual or unit or accurate" > gpurun_out/r4e/tests_pipe2.log 2>&1 || { echo PIPE2_FAILED; tail -30 gpurun_out/r4e/tests_pipe2.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_engine.py tests/test_gemm.py tests/test_transformer.py tests/test_im2col.py > gpurun_out/r4e/tests2.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r4e/tests2.log; exit 1; }
for f in b20_5 b200_50 b200_50_nopipe b20_5_notape; do python -c "import json,sys; r=json.loads(open('gpurun_out/r4e/$f.log').read().strip().splitlines()[-1]); print('$f', r['value'], r['ms_per_step'], r['host_enqueue_ms_per_step'])"; done

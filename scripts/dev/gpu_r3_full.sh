#!/bin/bash
# round-3 full GPU validation: gpu test suite, smoke, 1-GPU bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3_full_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r3_full_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r3_smoke.log 2>&1 || exit $?
tail -2 gpurun_out/r3_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3_bench_final.log 2>&1 || exit $?
tail -1 gpurun_out/r3_bench_final.log

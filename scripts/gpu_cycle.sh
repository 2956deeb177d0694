#!/bin/bash
# One build-measure cycle on the GPU box: selected GPU tests, the 1-GPU bench,
# and a kernel-trace round split (scripts/round_kernels.py).  Each GPU step has
# its own time limit; any failure stops the script.
#   TESTS="tests/test_sketch_region.py" MARKER=cs_region_encode bash scripts/gpu_cycle.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-cyc}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_bench.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$MARKER" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_rp -o bench \
    -- python3 bench.py --steps 30 --warmup 10 $BENCH_ARGS > gpurun_out/${TAG}_rp.log 2>&1 || exit $?
  python scripts/round_kernels.py gpurun_out/${TAG}_rp/bench_kernel_trace.csv --marker "$MARKER" \
    --rounds 8 > gpurun_out/${TAG}_rk.txt
  head -${RK_LINES:-30} gpurun_out/${TAG}_rk.txt
  rm -f gpurun_out/${TAG}_rp/bench_kernel_trace.csv.gz
fi

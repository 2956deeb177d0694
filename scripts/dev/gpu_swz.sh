# halo window swizzle: conv tests + alternating bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/swz_tests.log 2>&1 || { tail -30 gpurun_out/swz_tests.log; exit 1; }
tail -1 gpurun_out/swz_tests.log
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 60 --warmup 10 | cut -c1-130 || exit 1
  COMMEFF_HALO_SWIZZLE=0 timeout -k 10 200 python3 bench.py --steps 60 --warmup 10 | cut -c1-130 || exit 1
done

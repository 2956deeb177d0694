set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
COMMEFF_HALO_PF=1 timeout -k 10 300 python -u -m pytest tests/test_conv.py -x -q -m gpu --timeout 250 --timeout-method thread > gpurun_out/r3_pytest_pf.log 2>&1 || { echo "pf tests failed"; tail -30 gpurun_out/r3_pytest_pf.log; exit 1; }
tail -1 gpurun_out/r3_pytest_pf.log
for pf in 0 1 0 1; do
  COMMEFF_HALO_PF=$pf timeout -k 10 200 python bench.py --steps 40 --warmup 5 > gpurun_out/r3_bench_pf$pf.log 2>&1
  echo "pf=$pf $(tail -1 gpurun_out/r3_bench_pf$pf.log | cut -c1-140)"
done
COMMEFF_HALO_PF=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_pf -o tr -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_pf.log 2>&1
python3 scripts/round_kernels.py $(find gpurun_out/prof_pf -name "*kernel_trace.csv" | head -1) --rounds 8 --top 12

cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5tn3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_fedavg_native.py tests/test_gemm.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 -1 0 1 -1 0; do
  if [ $v = 0 ]; then export COMMEFF_FA_TN=0; else export COMMEFF_FA_TN=1 COMMEFF_FA_TN_SMALL=$v; fi
  timeout -k 10 300 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 5 --warmup 2 > $O/tn$v.log 2>&1 || { tail -20 $O/tn$v.log; exit 1; }
  echo "small=$v: $(tail -1 $O/tn$v.log | cut -c1-110)"
done
export COMMEFF_FA_TN=1 COMMEFF_FA_TN_SMALL=1
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o run -- python scripts/bench_configs.py --config cifar100_fedavg_local --steps 2 --warmup 1 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }

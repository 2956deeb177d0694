cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5imps; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_fedavg_native.py tests/test_gemm.py tests/test_im2col.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 1 0 1 0 1 0; do
  AB_IMPS=$v timeout -k 10 300 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 8 --warmup 2 > $O/b$v.log 2>&1 || { tail -20 $O/b$v.log; exit 1; }
  echo "imps=$v: $(tail -1 $O/b$v.log | cut -c60-110)"
done

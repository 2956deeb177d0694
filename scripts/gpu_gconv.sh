# grouped (channel-stacked) conv kernels for batched FedAvg: tests + bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4x}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv.py -k "grouped" > $O/gconv_tests.log 2>&1 || { echo GCONV_TESTS_FAILED; tail -40 $O/gconv_tests.log; exit 1; }
tail -1 $O/gconv_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fedavg_batched.py > $O/fedavg_tests.log 2>&1 || { echo FEDAVG_TESTS_FAILED; tail -40 $O/fedavg_tests.log; exit 1; }
tail -1 $O/fedavg_tests.log
for v in 1 0; do
  COMMEFF_GCONV=$v timeout -k 10 400 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 4 --warmup 2 > $O/fedavg_g$v.log 2>&1 || { tail -20 $O/fedavg_g$v.log; exit 1; }
  echo "fedavg gconv=$v: $(tail -1 $O/fedavg_g$v.log | cut -c1-230)"
done

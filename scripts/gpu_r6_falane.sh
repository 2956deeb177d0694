# native FedAvg engines with the weight updates on the side lane: tests, then
# the two FedAvg configs alternating COMMEFF_CONV_LANE=1/0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6falane}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_fedavg_native.py tests/test_fedavg_batched.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for c in cifar100_fedavg_local cifar10_resnet9_fedavg_local; do
    for v in 1 0; do
      COMMEFF_CONV_LANE=$v timeout -k 10 300 python scripts/bench_configs.py --config $c --steps 6 --warmup 2 > $O/${c}_${v}_$r.log 2>&1 || { tail -20 $O/${c}_${v}_$r.log; exit 1; }
      echo "lane=$v $c $(tail -1 $O/${c}_${v}_$r.log | grep -o '"value": [0-9.]*\|"ms_per_round": [0-9.]*' | tr '\n' ' ')"
    done
  done
done

# native batched FedAvg: kernel + engine tests, then the local-SGD bench (native vs vmap)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5fa}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_fedavg_native.py "tests/test_ops.py::test_client_tail_matches_composition" > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 5 --warmup 2 > $O/fa_native.log 2>&1 || { tail -30 $O/fa_native.log; exit 1; }
tail -1 $O/fa_native.log
timeout -k 10 300 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 5 --warmup 2 -- --fedavg_engine vmap > $O/fa_vmap.log 2>&1 || { tail -30 $O/fa_vmap.log; exit 1; }
tail -1 $O/fa_vmap.log

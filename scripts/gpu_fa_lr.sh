cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4falr}
mkdir -p $O
timeout -k 10 500 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 20 --warmup 3 > $O/fa.log 2>&1 || { tail -20 $O/fa.log; exit 1; }
tail -1 $O/fa.log | cut -c1-300

# native batched FedAvg: kernel-time profile + host sync points of the local-SGD bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5faprof}
mkdir -p $O
COMMEFF_SYNC_DEBUG=1 timeout -k 10 300 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 2 --warmup 1 > $O/sync.log 2>&1 || { tail -30 $O/sync.log; exit 1; }
grep -c SYNC $O/sync.log || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python scripts/bench_configs.py --config cifar100_fedavg_local --steps 3 --warmup 1 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
tail -1 $O/prof.log
find $O/prof -name "*kernel_stats.csv" | head -3

cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5src2; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o run -- python scripts/bench_configs.py --config cifar100_fedavg_local --steps 2 --warmup 1 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }

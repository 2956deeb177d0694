# batched FedAvg (5 local steps): bench, host profile, kernel split
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4r}
mkdir -p $O
timeout -k 10 400 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 4 --warmup 2 > $O/fedavg.log 2>&1 || { tail -20 $O/fedavg.log; exit 1; }
tail -1 $O/fedavg.log | cut -c1-300
COMMEFF_PROFILE_ROUNDS=$O/hp_rounds.txt timeout -k 10 400 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 3 --warmup 2 > $O/hp.log 2>&1 || { tail -20 $O/hp.log; exit 1; }
head -45 $O/hp_rounds.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o bench -- python3 scripts/bench_configs.py --config cifar100_fedavg_local --steps 2 --warmup 1 > $O/rp.log 2>&1 || exit 1
python scripts/round_kernels.py $O/rp/bench_kernel_trace.csv --tail-ms 300 --rounds 1 --top 30 > $O/rk.txt 2>&1
head -34 $O/rk.txt
rm -f $O/rp/bench_kernel_trace.csv

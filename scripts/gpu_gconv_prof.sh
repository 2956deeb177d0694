# batched FedAvg kernel split with / without the grouped native convs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4y}
mkdir -p $O
for v in 1 0; do
  COMMEFF_GCONV=$v timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp$v -o bench -- python3 scripts/bench_configs.py --config cifar100_fedavg_local --steps 2 --warmup 1 > $O/rp$v.log 2>&1 || exit 1
  python scripts/round_kernels.py $O/rp$v/bench_kernel_trace.csv --tail-ms 185 --rounds 1 --top 25 > $O/rk$v.txt 2>&1
  echo "== gconv=$v"; head -28 $O/rk$v.txt | cut -c1-150
  rm -f $O/rp$v/bench_kernel_trace.csv
done

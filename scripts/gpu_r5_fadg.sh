cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5fadg; mkdir -p $O
for w in 1 8 16 1 8 16; do
  COMMEFF_FA_DGRAD_W=$w timeout -k 10 300 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 5 --warmup 2 > $O/w$w.log 2>&1 || { tail -20 $O/w$w.log; exit 1; }
  echo "W>=$w: $(tail -1 $O/w$w.log | cut -c1-120)"
done

cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5ww; mkdir -p $O
for v in 16 32 64 16 32 64; do
  AB_WW=$v timeout -k 10 300 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 8 --warmup 2 > $O/b$v.log 2>&1 || { tail -20 $O/b$v.log; exit 1; }
  echo "halo_w>=$v: $(tail -1 $O/b$v.log | cut -c60-110)"
done

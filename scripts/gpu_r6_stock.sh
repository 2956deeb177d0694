# call sites of stock kernels / device allocations in a config's rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6stock}; mkdir -p $O
for c in ${CONFIGS:-imagenet_local_topk}; do
  COMMEFF_STOCK_SITES=$O/sites_$c.txt timeout -k 10 500 python scripts/bench_configs.py --config $c --steps ${STEPS:-6} --warmup 2 > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  tail -1 $O/$c.log | cut -c1-400
  head -30 $O/sites_$c.txt
done

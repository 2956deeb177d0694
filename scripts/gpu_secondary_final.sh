# secondary BASELINE configs on the final tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4sec}
mkdir -p $O
for c in gpt2_sketch cifar100_fedavg cifar100_fedavg_local imagenet_local_topk; do
  timeout -k 10 500 python scripts/bench_configs.py --config $c --steps 10 --warmup 3 > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  echo "$c: $(tail -1 $O/$c.log | cut -c1-300)"
done

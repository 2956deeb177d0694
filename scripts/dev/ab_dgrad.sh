cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5nt; mkdir -p $O
for v in 0 1 0 1 0 1; do
  if [ $v = 1 ]; then export AB_NT=1; else unset AB_NT; fi
  timeout -k 10 300 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 8 --warmup 2 > $O/b$v.log 2>&1 || { tail -20 $O/b$v.log; exit 1; }
  echo "nt=$v: $(tail -1 $O/b$v.log | cut -c60-110)"
done

cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_cfg
for c in imagenet_local_topk gpt2_sketch cifar100_fedavg; do
  echo "=== $c"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg/$c -o k --output-format csv -- python3 scripts/bench_configs.py --config $c --steps 3 --warmup 2 > gpurun_out/prof_cfg/$c.log 2>&1
  rc=$?; echo rc=$rc; tail -3 gpurun_out/prof_cfg/$c.log
  case $rc in 124|134|137|139) exit $rc;; esac
done

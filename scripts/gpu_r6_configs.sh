# the secondary BASELINE configs (bench_configs.py) and a GPT-2 round kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6cfg}; mkdir -p $O
: > $O/configs.jsonl
for c in ${CONFIGS:-gpt2_sketch imagenet_local_topk cifar100_fedavg_local}; do
  timeout -k 10 400 python scripts/bench_configs.py --config $c --steps 8 --warmup 2 > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  tail -1 $O/$c.log >> $O/configs.jsonl
  echo "$c: $(tail -1 $O/$c.log | cut -c1-220)"
done
if [ -n "${TRACE:-gpt2_sketch}" ]; then
  c=${TRACE:-gpt2_sketch}
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 scripts/bench_configs.py --config $c --steps 4 --warmup 2 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
  python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --tail-ms ${TAILMS:-50} --rounds 3 --top 60 > $O/rk_$c.txt 2>&1
  rm -f $O/rp/tr_kernel_trace.csv
  head -45 $O/rk_$c.txt
fi

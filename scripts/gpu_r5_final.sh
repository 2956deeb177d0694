# round-5 final tree on one box: driver-shaped headline bench, the three other
# BASELINE configs, and the ImageNet round's kernel table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5final}
mkdir -p $O
: > $O/final.jsonl
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log >> $O/final.jsonl
for c in cifar100_fedavg_local imagenet_local_topk gpt2_sketch; do
  timeout -k 10 400 python scripts/bench_configs.py --config $c --steps 8 --warmup 2 > $O/$c.log 2>&1 || { tail -20 $O/$c.log; exit 1; }
  tail -1 $O/$c.log >> $O/final.jsonl
  echo "$c: $(tail -1 $O/$c.log | cut -c1-160)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 scripts/bench_configs.py --config imagenet_local_topk --steps 4 --warmup 2 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --tail-ms 150 --rounds 3 --top 80 > $O/rk_imagenet.txt 2>&1
head -30 $O/rk_imagenet.txt
rm -f $O/rp/tr_kernel_trace.csv

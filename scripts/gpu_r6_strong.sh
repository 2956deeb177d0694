# strong-scaling rehearsal on one GPU: the per-rank round of a W = 100 round at N = 1/2/4/8
# (100 / 50 / 25 / 13 clients), a kernel trace of the 13-client round, and an ImageNet trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6strong}; mkdir -p $O
: > $O/strong.jsonl
for w in 100 50 25 13; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 20 --clients-per-round $w > $O/b_$w.log 2>&1 || { tail -20 $O/b_$w.log; exit 1; }
  tail -1 $O/b_$w.log >> $O/strong.jsonl
  python -c "import json; r=json.loads(open('$O/b_$w.log').read().strip().splitlines()[-1]); print('W=$w', r['value'], r['ms_per_step'], r['scaling'], r['host_enqueue_ms_per_step'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 bench.py --steps 20 --warmup 5 --clients-per-round 13 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --marker augment_kernel --rounds 12 --sequence --top 60 > $O/seq13.txt 2>&1
rm -f $O/rp/tr_kernel_trace.csv
head -3 $O/seq13.txt; grep "rounds=" $O/seq13.txt
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rpi -o tr -- python3 scripts/bench_configs.py --config imagenet_local_topk --steps 4 --warmup 2 > $O/rpi.log 2>&1 || { tail -20 $O/rpi.log; exit 1; }
python scripts/round_kernels.py $O/rpi/tr_kernel_trace.csv --tail-ms 150 --rounds 3 --top 80 > $O/rk_imagenet.txt 2>&1
rm -f $O/rpi/tr_kernel_trace.csv
head -60 $O/rk_imagenet.txt

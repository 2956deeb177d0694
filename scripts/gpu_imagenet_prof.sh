# ImageNet ResNet-101 local top-k round: bench + per-round kernel table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4in}
mkdir -p $O
timeout -k 10 400 python scripts/bench_configs.py --config imagenet_local_topk --steps 6 --warmup 2 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 scripts/bench_configs.py --config imagenet_local_topk --steps 4 --warmup 2 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --tail-ms ${TAILMS:-150} --rounds 3 --top 80 > $O/rk.txt 2>&1
head -60 $O/rk.txt
rm -f $O/rp/tr_kernel_trace.csv

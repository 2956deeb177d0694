# GPT-2 round of the final tree: kernel sequence (both streams) and per-kernel totals
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6g2tr}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 scripts/bench_configs.py --config gpt2_sketch --steps 6 --warmup 3 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --marker cs_region_encode --rounds 3 --top 60 > $O/top.txt 2>&1
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --marker cs_region_encode --rounds 3 --top 5 --sequence > $O/seq.txt 2>&1
rm -f $O/rp/tr_kernel_trace.csv
head -40 $O/top.txt | cut -c1-150

# GPT-2 round: kernel sequence with workgroup counts, plus the isolated GEMM micro-benchmark
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6g2seq}; mkdir -p $O
timeout -k 10 300 python scripts/bench_gemm.py > $O/gemm.jsonl 2>&1 || { tail -20 $O/gemm.jsonl; exit 1; }
cut -c1-200 $O/gemm.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 scripts/bench_configs.py --config gpt2_sketch --steps 5 --warmup 2 ${EXTRA:-} > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --marker cs_region_encode --rounds 3 --top 50 --sequence > $O/seq.txt 2>&1
rm -f $O/rp/tr_kernel_trace.csv
tail -52 $O/seq.txt

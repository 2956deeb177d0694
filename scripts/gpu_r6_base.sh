# round-6 baseline: driver-shaped headline bench, isolated conv layer timings and one
# traced round's kernels in launch order
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6base}; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
tail -1 $O/b.log | cut -c1-200
timeout -k 10 200 python scripts/dev/conv_lab.py > $O/lab.log 2>&1 || { tail -20 $O/lab.log; exit 1; }
tail -1 $O/lab.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 bench.py --steps 20 --warmup 5 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --marker augment_kernel --rounds 12 --sequence --top 60 > $O/seq.txt 2>&1
rm -f $O/rp/tr_kernel_trace.csv
head -70 $O/seq.txt
timeout -k 10 200 python scripts/bench_gemm_tn.py > $O/tn.log 2>&1 || { tail -20 $O/tn.log; exit 1; }
cat $O/tn.log

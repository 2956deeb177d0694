# kernel trace of the 13-client round (strong-scaling per-rank share at N = 8)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6t13}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 bench.py --steps 20 --warmup 5 --clients-per-round ${W:-13} > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --marker augment_kernel --rounds 12 --sequence --top 60 > $O/seq.txt 2>&1
rm -f $O/rp/tr_kernel_trace.csv
head -60 $O/seq.txt

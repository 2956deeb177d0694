# bench A/B: streamed conv kernel on/off (alternating), + kernel trace of the stream round
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5ab}
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    COMMEFF_CONV_STREAM=$v timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b_${v}_$r.log 2>&1 || { tail -20 $O/b_${v}_$r.log; exit 1; }
    python -c "import json,sys; r=json.loads(open('$O/b_${v}_$r.log').read().strip().splitlines()[-1]); print('stream=$v', r['value'], r['ms_per_step'], r['weights_checksum'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o bench -- python3 bench.py --steps 60 --warmup 20 > $O/rp.log 2>&1 || exit 1
python scripts/round_kernels.py $O/rp/bench_kernel_trace.csv --marker cs_region_encode --rounds 30 --gaps 6 --top 40 > $O/rk.txt 2>&1
head -40 $O/rk.txt
rm -f $O/rp/bench_kernel_trace.csv

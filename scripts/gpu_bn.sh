# ghost BN micro-benchmark (+ per-kernel stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4bn}
mkdir -p $O
timeout -k 10 300 python scripts/bench_bn.py > $O/bn.log 2>&1 || { tail -20 $O/bn.log; exit 1; }
cat $O/bn.log
if [ -n "$STATS" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp -o bn -- python3 scripts/bench_bn.py --iters 5 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
find $O/rp -name "*kernel_stats.csv" -exec cp {} $O/kstats.csv \;
python -c "
import csv
for r in csv.DictReader(open('$O/kstats.csv')):
    if 'bn_' in r['Name']: print(r['Name'][:60], r['Calls'], r['TotalDurationNs'], r['AverageNs'])
"
find $O/rp -name "*kernel_trace.csv" -delete
fi

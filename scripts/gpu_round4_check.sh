# round-4 GPU check: benches first (kept even if a test fails), a per-round
# kernel trace of the driver-shaped bench, then the GPU test suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4f}
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --round-times > $O/b20_5.log 2>&1 || { tail -20 $O/b20_5.log; exit 1; }
COMMEFF_TAPE=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --round-times > $O/b20_5_notape.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b200_50.log 2>&1 || exit 1
COMMEFF_TAPE=0 timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b200_50_notape.log 2>&1 || exit 1
for f in b20_5 b20_5_notape b200_50 b200_50_notape; do python -c "import json,sys; r=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', r['value'], r['ms_per_step'], r['host_enqueue_ms_per_step'], r.get('round_ms'))"; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o bench -- python3 bench.py --steps 20 --warmup 5 > $O/rp.log 2>&1 || exit 1
python scripts/round_kernels.py $O/rp/bench_kernel_trace.csv --marker cs_region_encode --rounds 8 --per-round 8 --top 60 > $O/rk.txt 2>&1
head -40 $O/rk.txt
rm -f $O/rp/bench_kernel_trace.csv
if [ -n "$SKIP_TESTS" ]; then exit 0; fi
timeout -k 10 1200 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log

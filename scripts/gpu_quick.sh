# quick check: tape / engine / transformer GPU tests, benches, round gaps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4w}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_tape.py tests/test_engine.py tests/test_transformer.py tests/test_drivers.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20_5_$r.log 2>&1 || { tail -20 $O/b20_5_$r.log; exit 1; }
  timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b200_50_$r.log 2>&1 || { tail -20 $O/b200_50_$r.log; exit 1; }
done
for f in b20_5_1 b200_50_1 b20_5_2 b200_50_2; do python -c "import json,sys; r=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', r['value'], r['ms_per_step'], r['host_enqueue_ms_per_step'], r['weights_checksum'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o bench -- python3 bench.py --steps 60 --warmup 20 > $O/rp.log 2>&1 || exit 1
python scripts/round_kernels.py $O/rp/bench_kernel_trace.csv --marker cs_region_encode --rounds 30 --gaps 6 --top 5 > $O/rk.txt 2>&1
head -14 $O/rk.txt
rm -f $O/rp/bench_kernel_trace.csv

# candidate top-k rewrite: region / top-k tests, then headline bench and GPT-2 config (2 each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6cand}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_sketch_region.py tests/test_sketch_plan.py tests/test_ops.py tests/test_engine.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_$r.log 2>&1 || { tail -20 $O/b_$r.log; exit 1; }
  python -c "import json; r=json.loads(open('$O/b_$r.log').read().strip().splitlines()[-1]); print('bench', r['value'], r['ms_per_step'])"
  timeout -k 10 300 python scripts/bench_configs.py --config gpt2_sketch --steps 8 --warmup 3 > $O/g_$r.log 2>&1 || { tail -20 $O/g_$r.log; exit 1; }
  python -c "import json; r=json.loads(open('$O/g_$r.log').read().strip().splitlines()[-1]); print('gpt2', r['value'], r['ms_per_round'])"
done
for c in "bench.py --steps 10 --warmup 3" "scripts/bench_configs.py --config gpt2_sketch --steps 4 --warmup 2"; do
  rm -rf $O/rp
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rp -o tr -- python3 $c > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
  python - $O/rp/tr_results.db <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
for key in ["cand_compact", "cand_scan", "write_kernel", "hist_kernel<1", "cs_region_query"]:
    print(key, [round((e - s) / 1e3, 1) for n, s, e in rows if key in n][-6:])
PY
done

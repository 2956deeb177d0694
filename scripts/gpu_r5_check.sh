# full GPU suite + driver-shaped benches (with per-round times)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5check}
mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --round-times > $O/b20_5_$r.log 2>&1 || { tail -20 $O/b20_5_$r.log; exit 1; }
  python -c "import json,sys; r=json.loads(open('$O/b20_5_$r.log').read().strip().splitlines()[-1]); print('20/5', r['value'], r['ms_per_step'], r['warmup_to_timed_ms'], r['round_ms'][:6])"
done

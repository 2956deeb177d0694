# full GPU suite (no -x: every failure listed) + driver-shaped benches (with per-round times)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5check}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1
rc=$?
tail -12 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "TESTS ABORTED rc=$rc"; exit 1; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --round-times > $O/b20_5_$r.log 2>&1 || { tail -20 $O/b20_5_$r.log; exit 1; }
  python -c "import json,sys; r=json.loads(open('$O/b20_5_$r.log').read().strip().splitlines()[-1]); print('20/5', r['value'], r['ms_per_step'], r['warmup_to_timed_ms'], r['round_ms'][:6])"
done
exit $rc

# driver-shaped bench (20 timed after 5) x3 with per-round times + the two-rank bench test
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4short}
mkdir -p $O
for r in 0 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --round-times > $O/b$r.log 2>&1 || { tail -20 $O/b$r.log; exit 1; }
  tail -1 $O/b$r.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['ms_per_step'], r['host_enqueue_ms_per_step'], r.get('barrier_before_timed_ms'), r['round_ms'][:6])"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_distributed.py -k bench > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log

# driver-shaped bench under a kernel trace: per-round timeline around the warmup -> timed boundary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5gap}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tape.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --round-times > $O/b$r.log 2>&1 || { tail -20 $O/b$r.log; exit 1; }
python -c "import json; r=json.loads(open('$O/b$r.log').read().strip().splitlines()[-1]); print('20/5', r['value'], r['ms_per_step'], r['warmup_to_timed_ms'], r['warmup_host_ms'], r['round_ms'][:6])"
done
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python scripts/dev/trace_gaps.py $O/prof/run_results.db > $O/gaps.txt && head -12 $O/gaps.txt

# A/B of an environment switch on a bench_configs.py configuration (alternating runs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6cfgab}; mkdir -p $O
VAR=${VAR:?set VAR to the switch under test}; VALS=${VALS:?set VALS}; C=${CONFIG:-gpt2_sketch}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for r in ${ROUNDS:-1 2}; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python scripts/bench_configs.py --config $C --steps ${STEPS:-8} --warmup 3 > $O/${v}_${r}.log 2>&1 || { tail -20 $O/${v}_${r}.log; exit 1; }
    python -c "import json; r=json.loads(open('$O/${v}_${r}.log').read().strip().splitlines()[-1]); print('$VAR=$v', r['value'], r['ms_per_round'])"
  done
done

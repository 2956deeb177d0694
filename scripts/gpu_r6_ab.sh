# A/B of an environment switch: conv tests, then conv_lab and the driver-shaped bench
# alternating over VALS of VAR (e.g. VAR=COMMEFF_FA_HEAD VALS="1 0")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6ab}; mkdir -p $O
VAR=${VAR:?set VAR to the switch under test}; VALS=${VALS:?set VALS}
if [ -n "${TESTS-tests/test_conv.py}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${TESTS-tests/test_conv.py} > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for r in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python ${MICRO:-scripts/dev/conv_lab.py} > $O/lab_${v}_${r}.log 2>&1 || { tail -20 $O/lab_${v}_${r}.log; exit 1; }
    echo "$VAR=$v lab: $(grep '^{' $O/lab_${v}_${r}.log | cut -c1-330)"
    env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_${v}_${r}.log 2>&1 || { tail -20 $O/b_${v}_${r}.log; exit 1; }
    python -c "import json; r=json.loads(open('$O/b_${v}_${r}.log').read().strip().splitlines()[-1]); print('$VAR=$v bench', r['value'], r['ms_per_step'])"
  done
done

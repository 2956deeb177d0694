# interleaved wgrad loops: numerics, per-layer timing, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4q}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv.py > $O/conv_tests.log 2>&1 || { echo CONV_TESTS_FAILED; tail -30 $O/conv_tests.log; exit 1; }
tail -1 $O/conv_tests.log
for il in 1 0; do
  COMMEFF_WGRAD_IL=$il timeout -k 10 200 python scripts/conv_ablate.py > $O/layers_il$il.log 2>&1 || { tail -5 $O/layers_il$il.log; exit 1; }
  echo "il=$il"; grep '^{' $O/layers_il$il.log
done
for il in 1 0 1 0; do
  COMMEFF_WGRAD_IL=$il timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b_il$il.log 2>&1 || { tail -20 $O/b_il$il.log; exit 1; }
  echo "bench il=$il $(tail -1 $O/b_il$il.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["weights_checksum"])')"
done

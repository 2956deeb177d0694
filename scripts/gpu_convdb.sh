# double-buffered halo conv loop: numerics, per-layer timing, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4o}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv.py > $O/conv_tests.log 2>&1 || { echo CONV_TESTS_FAILED; tail -30 $O/conv_tests.log; exit 1; }
tail -1 $O/conv_tests.log
for db in 1 0; do
  COMMEFF_CONV_DB=$db timeout -k 10 200 python scripts/conv_ablate.py > $O/layers_db$db.log 2>&1 || { tail -5 $O/layers_db$db.log; exit 1; }
  echo "db=$db"; grep '^{' $O/layers_db$db.log
done
for db in 1 0 1 0; do
  COMMEFF_CONV_DB=$db timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b_db$db.log 2>&1 || { tail -20 $O/b_db$db.log; exit 1; }
  echo "bench db=$db $(tail -1 $O/b_db$db.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["weights_checksum"])')"
done

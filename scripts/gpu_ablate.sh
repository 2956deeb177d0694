# halo conv forward ablations (timing only) + the tape tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4i}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_tape.py tests/test_conv.py -k "tape or taped or deferred" > $O/tape_tests.log 2>&1 || { echo TAPE_TESTS_FAILED; tail -30 $O/tape_tests.log; exit 1; }
tail -1 $O/tape_tests.log
for ab in 0 1 2 4 3 7; do
  COMMEFF_CONV_ABLATE=$ab timeout -k 10 200 python scripts/conv_ablate.py > $O/ablate_$ab.log 2>&1 || { tail -5 $O/ablate_$ab.log; exit 1; }
  grep '^{' $O/ablate_$ab.log
done

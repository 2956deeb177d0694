cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5mp; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_im2col.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python scripts/dev/bench_maxpool.py

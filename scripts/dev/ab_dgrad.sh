cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5rowsgd; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_fedavg_batched.py > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/tests.log; exit 1; }
tail -6 $O/tests.log

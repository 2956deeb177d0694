# full GPU suite (no -x: every failure listed), then the driver-shaped headline bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6tests}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/ ${TESTS:-} > $O/tests.log 2>&1
rc=$?
tail -15 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "TESTS ABORTED rc=$rc"; exit 1; }
exit $rc

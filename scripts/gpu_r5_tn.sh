cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5tn; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo deep; timeout -k 10 200 python scripts/bench_gemm_tn.py > $O/deep.log 2>&1 || { tail -20 $O/deep.log; exit 1; }; cat $O/deep.log
echo old; COMMEFF_TN_DEEP=0 timeout -k 10 200 python scripts/bench_gemm_tn.py > $O/old.log 2>&1 || { tail -20 $O/old.log; exit 1; }; cat $O/old.log

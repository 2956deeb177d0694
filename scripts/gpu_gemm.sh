# native GEMM kernels: numerics tests, micro-benchmark (big vs 128-row vs hipBLASLt), GPT-2 round
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4j}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm.py > $O/gemm_tests.log 2>&1 || { echo GEMM_TESTS_FAILED; tail -30 $O/gemm_tests.log; exit 1; }
tail -1 $O/gemm_tests.log
timeout -k 10 300 python scripts/bench_gemm.py > $O/gemm_big.log 2>&1 || { tail -20 $O/gemm_big.log; exit 1; }
cat $O/gemm_big.log | grep '^{'
COMMEFF_GEMM_BIG=0 timeout -k 10 300 python scripts/bench_gemm.py > $O/gemm_small.log 2>&1 || { tail -20 $O/gemm_small.log; exit 1; }
cat $O/gemm_small.log | grep '^{' | cut -c1-120
for g in native blas; do
  COMMEFF_GEMM=$g timeout -k 10 400 python scripts/bench_configs.py --config gpt2_sketch --steps 20 --warmup 5 > $O/gpt2_$g.log 2>&1 || { tail -20 $O/gpt2_$g.log; exit 1; }
  echo "gpt2 $g: $(tail -1 $O/gpt2_$g.log | cut -c1-200)"
done

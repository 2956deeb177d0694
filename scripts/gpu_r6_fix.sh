# split-K fix-up: TN GEMM tests, isolated TN timings and the GPT-2 round, A/B vs the reduce kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6fix}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests/test_gemm_tn.py} > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in 0 1; do
  COMMEFF_SPLITK_FIX=$v timeout -k 10 200 python scripts/bench_gemm_tn.py > $O/tn_$v.log 2>&1 || { tail -20 $O/tn_$v.log; exit 1; }
  echo "FIX=$v"; cat $O/tn_$v.log | grep '^{'
done
for r in 1 2; do
  for v in 0 1; do
    COMMEFF_SPLITK_FIX=$v timeout -k 10 400 python scripts/bench_configs.py --config ${CONFIG:-gpt2_sketch} --steps 10 --warmup 3 > $O/cfg_${v}_$r.log 2>&1 || { tail -20 $O/cfg_${v}_$r.log; exit 1; }
    echo "FIX=$v: $(tail -1 $O/cfg_${v}_$r.log | cut -c1-200)"
  done
done

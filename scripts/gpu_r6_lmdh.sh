# native split-K dh of the tied LM head: GEMM / transformer tests, GPT-2 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6lmdh}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gemm.py tests/test_transformer.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in native blas; do
    COMMEFF_LM_DH=$v timeout -k 10 300 python scripts/bench_configs.py --config gpt2_sketch --steps 8 --warmup 3 > $O/g2_${v}_$r.log 2>&1 || { tail -20 $O/g2_${v}_$r.log; exit 1; }
    echo "dh=$v $(tail -1 $O/g2_${v}_$r.log | grep -o '"ms_per_round": [0-9.]*\|"value": [0-9.]*' | tr '\n' ' ')"
  done
done

# GPT-2 side-stream column sums: tests + bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4t}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transformer.py tests/test_drivers.py -m gpu > $O/tx_tests.log 2>&1 || { echo TX_TESTS_FAILED; tail -30 $O/tx_tests.log; exit 1; }
tail -1 $O/tx_tests.log
for v in 1 0 1 0; do
  COMMEFF_COLSUM_SIDE=$v timeout -k 10 400 python scripts/bench_configs.py --config gpt2_sketch --steps 30 --warmup 5 > $O/gpt2_cs$v.log 2>&1 || { tail -20 $O/gpt2_cs$v.log; exit 1; }
  echo "gpt2 colsum_side=$v: $(tail -1 $O/gpt2_cs$v.log | cut -c1-200)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp_gpt2 -o bench -- python3 scripts/bench_configs.py --config gpt2_sketch --steps 12 --warmup 4 > $O/rp_gpt2.log 2>&1 || exit 1
python scripts/round_kernels.py $O/rp_gpt2/bench_kernel_trace.csv --marker cs_region_encode --rounds 8 --gaps 10 --top 30 > $O/rk_gpt2.txt 2>&1
head -45 $O/rk_gpt2.txt
rm -f $O/rp_gpt2/bench_kernel_trace.csv

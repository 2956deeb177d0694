cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5g2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_transformer.py tests/test_drivers.py tests/test_ops.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python scripts/bench_configs.py --config gpt2_sketch --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/prof -o run -- python scripts/bench_configs.py --config gpt2_sketch --steps 3 --warmup 1 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python scripts/dev/rocpd_top.py $O/prof/run_results.db 4 60 > $O/top.txt && grep -i "native\|Cijk\|rocprim\|embed\|ce_fwd\|scale_rows" $O/top.txt | head -30

# native tied LM head: tests, GPT-2 bench, round kernel split (no hipBLASLt left?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4lm}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_transformer.py tests/test_drivers.py tests/test_gemm.py -k "lm_head or gpt2_driver or tn" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 400 python scripts/bench_configs.py --config gpt2_sketch --steps 20 --warmup 5 > $O/gpt2.log 2>&1 || { tail -20 $O/gpt2.log; exit 1; }
echo "gpt2: $(tail -1 $O/gpt2.log | cut -c1-250)"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o bench -- python3 scripts/bench_configs.py --config gpt2_sketch --steps 12 --warmup 4 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/bench_kernel_trace.csv --marker cs_region_encode --rounds 8 --gaps 8 --top 60 > $O/rk.txt 2>&1
head -45 $O/rk.txt
grep -c Cijk $O/rk.txt || true
rm -f $O/rp/bench_kernel_trace.csv

# LM head dW on the native TN GEMM vs hipBLASLt (side lane), then the kernels
# of a GPT-2 round that are not native (hipBLASLt / stock) with both native
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6lmdw}; mkdir -p $O
for r in 1 2; do
  for v in tn blas; do
    COMMEFF_LM_DW=$v timeout -k 10 300 python scripts/bench_configs.py --config gpt2_sketch --steps 8 --warmup 3 > $O/g2_${v}_$r.log 2>&1 || { tail -20 $O/g2_${v}_$r.log; exit 1; }
    echo "dw=$v $(tail -1 $O/g2_${v}_$r.log | grep -o '"ms_per_round": [0-9.]*\|"value": [0-9.]*' | tr '\n' ' ')"
  done
done
COMMEFF_LM_DW=tn timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 scripts/bench_configs.py --config gpt2_sketch --steps 4 --warmup 2 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --marker cs_region_encode --rounds 3 --top 80 > $O/top.txt 2>&1
rm -f $O/rp/tr_kernel_trace.csv
grep -a "Cijk\|at::native\|rocprim\|SoftMax" $O/top.txt | cut -c1-140 || true

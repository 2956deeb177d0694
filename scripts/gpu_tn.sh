# grouped TN GEMM tests + ImageNet round with the native 1x1 weight gradients
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4tn}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm.py tests/test_im2col.py tests/test_transformer.py -k "gemm_tn or tn_grouped or wgrad_native or tn_parts or im2col or col or 1x1" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -3 $O/t.log
for g in native blas; do
  COMMEFF_GEMM=$g timeout -k 10 400 python scripts/bench_configs.py --config imagenet_local_topk --steps 6 --warmup 2 > $O/imagenet_$g.log 2>&1 || { tail -20 $O/imagenet_$g.log; exit 1; }
  echo "imagenet $g: $(tail -1 $O/imagenet_$g.log | cut -c1-250)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 scripts/bench_configs.py --config imagenet_local_topk --steps 4 --warmup 2 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --tail-ms ${TAILMS:-150} --rounds 3 --top 80 > $O/rk.txt 2>&1
head -40 $O/rk.txt
rm -f $O/rp/tr_kernel_trace.csv

# BN statistics from the GEMM epilogue: tests, ImageNet A/B, round kernel split
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4bnepi}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bn_epi.py tests/test_gemm.py tests/test_conv.py -k "bn or bnstats or gemm or ghost" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 0 1; do for m in 1 0; do
  COMMEFF_BN_EPI=$m timeout -k 10 400 python scripts/bench_configs.py --config imagenet_local_topk --steps 8 --warmup 2 > $O/in_${m}_$r.log 2>&1 || { tail -20 $O/in_${m}_$r.log; exit 1; }
  echo "epi=$m run $r: $(tail -1 $O/in_${m}_$r.log | cut -c1-220)"
done; done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 scripts/bench_configs.py --config imagenet_local_topk --steps 4 --warmup 2 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --tail-ms ${TAILMS:-150} --rounds 3 --top 80 > $O/rk.txt 2>&1
head -30 $O/rk.txt
rm -f $O/rp/tr_kernel_trace.csv

# secondary configs (native MFMA GEMM vs hipBLASLt), GPT-2 round trace with
# idle-gap analysis, GPT-2 learning curve, convergence pin (region vs csvec)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4s}
mkdir -p $O
for g in native blas; do
  COMMEFF_GEMM=$g timeout -k 10 400 python scripts/bench_configs.py --config gpt2_sketch --steps 20 --warmup 5 > $O/gpt2_$g.log 2>&1 || { tail -20 $O/gpt2_$g.log; exit 1; }
  echo "gpt2 $g: $(tail -1 $O/gpt2_$g.log | cut -c1-300)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp_gpt2 -o bench -- python3 scripts/bench_configs.py --config gpt2_sketch --steps 12 --warmup 4 > $O/rp_gpt2.log 2>&1 || exit 1
python scripts/round_kernels.py $O/rp_gpt2/bench_kernel_trace.csv --marker cs_region_encode --rounds 8 --gaps 16 --top 50 > $O/rk_gpt2.txt 2>&1
head -70 $O/rk_gpt2.txt
rm -f $O/rp_gpt2/bench_kernel_trace.csv
for g in native blas; do
  COMMEFF_GEMM=$g timeout -k 10 400 python scripts/bench_configs.py --config imagenet_local_topk --steps 6 --warmup 2 > $O/imagenet_$g.log 2>&1 || { tail -20 $O/imagenet_$g.log; exit 1; }
  echo "imagenet $g: $(tail -1 $O/imagenet_$g.log | cut -c1-300)"
done
if [ -z "$SKIP_LONG" ]; then
timeout -k 10 600 python -u scripts/gpt2_learning.py --rounds 200 --every 20 --lr 0.3 --out $O/gpt2_learning.jsonl > $O/gpt2_learning.log 2>&1 || { tail -20 $O/gpt2_learning.log; exit 1; }
tail -3 $O/gpt2_learning.log
timeout -k 10 1500 python -u scripts/convergence.py --modes sketch@0.4,sketch_planned@0.4,sketch@0.1,sketch_planned@0.1,uncompressed@0.1 --out $O/convergence.jsonl > $O/convergence.log 2>&1 || { tail -20 $O/convergence.log; exit 1; }
grep CONVERGENCE $O/convergence.log
fi

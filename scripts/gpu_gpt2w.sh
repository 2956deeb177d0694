# GPT-2 round with the record worker processes vs inline record assembly
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4s2}
mkdir -p $O
for v in w2 w0 w2 w0; do
  if [ $v = w0 ]; then X="-- --train_dataloader_workers 0"; else X=""; fi
  timeout -k 10 400 python scripts/bench_configs.py --config gpt2_sketch --steps 30 --warmup 5 $X > $O/gpt2_$v.log 2>&1 || { tail -20 $O/gpt2_$v.log; exit 1; }
  echo "gpt2 $v: $(tail -1 $O/gpt2_$v.log | cut -c1-220)"
done

# full-size GPT-2 (12 x 768) FetchSGD learning curves on the learnable bigram text, a few LRs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6g2learn}; mkdir -p $O
: > $O/curves.jsonl
for lr in ${LRS:-0.02 0.05 0.1}; do
  timeout -k 10 400 python -u scripts/gpt2_learning.py --size small --rounds ${ROUNDS:-150} --every 25 --lr $lr --out $O/curves.jsonl > $O/lr_$lr.log 2>&1 || { tail -20 $O/lr_$lr.log; exit 1; }
  echo "lr $lr:"; grep '^{' $O/lr_$lr.log | python -c "import json,sys; [print(' ', {k: (round(v,3) if isinstance(v,float) else v) for k,v in json.loads(l).items()}) for l in sys.stdin]"
done

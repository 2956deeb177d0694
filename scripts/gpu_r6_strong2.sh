# strong-scaling rehearsal on one GPU with the side lane: the per-rank round of a
# W = 100 round at N = 1/2/4/8 (100 / 50 / 25 / 13 clients), lane on and off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6strong2}; mkdir -p $O
: > $O/strong.jsonl
for w in 100 50 25 13; do
  for v in 1 0; do
    COMMEFF_CONV_LANE=$v timeout -k 10 300 python bench.py --steps 50 --warmup 20 --clients-per-round $w > $O/b_${w}_$v.log 2>&1 || { tail -20 $O/b_${w}_$v.log; exit 1; }
    [ $v = 1 ] && tail -1 $O/b_${w}_$v.log >> $O/strong.jsonl
    python -c "import json; r=json.loads(open('$O/b_${w}_$v.log').read().strip().splitlines()[-1]); print('W=$w lane=$v', r['value'], r['ms_per_step'])"
  done
done

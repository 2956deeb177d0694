# bench A/B over the epilogue kinds the streamed conv kernel serves
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5ab2}
mkdir -p $O
for r in 1 2; do
  for v in 0 1 3 7 11 19 35 63; do
    COMMEFF_STREAM_EPI=$v timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b_${v}_$r.log 2>&1 || { tail -20 $O/b_${v}_$r.log; exit 1; }
    python -c "import json,sys; r=json.loads(open('$O/b_${v}_$r.log').read().strip().splitlines()[-1]); print('epi=$v', r['value'], r['ms_per_step'])"
  done
done

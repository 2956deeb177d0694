cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5split; mkdir -p $O
for v in 1 2 1 2 1 2; do
  AB_SPLITDIV=$v timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b$v.log 2>&1 || { tail -20 $O/b$v.log; exit 1; }
  python -c "import json; r=json.loads(open('$O/b$v.log').read().strip().splitlines()[-1]); print('div=$v', r['value'], r['ms_per_step'])"
done

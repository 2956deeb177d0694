# region-sketch query with several blocks per group at one rank
# (COMMEFF_QUERY_BPG): sketch tests with the override, GPT-2 and headline A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6qbpg}; mkdir -p $O
COMMEFF_QUERY_BPG=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_sketch_region.py tests/test_tape.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 0 2 4 0 2 4; do
  COMMEFF_QUERY_BPG=$v timeout -k 10 300 python scripts/bench_configs.py --config gpt2_sketch --steps 8 --warmup 3 > $O/g2_$v.log 2>&1 || { tail -20 $O/g2_$v.log; exit 1; }
  echo "bpg=$v gpt2 $(tail -1 $O/g2_$v.log | grep -o '"ms_per_round": [0-9.]*')"
  COMMEFF_QUERY_BPG=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_$v.log 2>&1 || { tail -20 $O/b_$v.log; exit 1; }
  python -c "import json; r=json.loads(open('$O/b_$v.log').read().strip().splitlines()[-1]); print('bpg=$v headline', r['value'], r['ms_per_step'])"
done

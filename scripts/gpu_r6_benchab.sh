# A/B of an environment switch on the driver-shaped headline bench only,
# alternating over VALS of VAR twice (e.g. VAR=COMMEFF_CONV_LANE VALS="1 0")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6benchab}; mkdir -p $O
VAR=${VAR:?set VAR to the switch under test}; VALS=${VALS:?set VALS}
for r in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_${v}_${r}.log 2>&1 || { tail -20 $O/b_${v}_${r}.log; exit 1; }
    python -c "import json; r=json.loads(open('$O/b_${v}_${r}.log').read().strip().splitlines()[-1]); print('$VAR=$v bench', r['value'], r['ms_per_step'])"
  done
done

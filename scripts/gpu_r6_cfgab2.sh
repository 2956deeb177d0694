# A/B of an environment switch on one bench_configs config (alternating, twice)
# e.g. CONFIG=imagenet_local_topk VAR=COMMEFF_BN_EPI VALS="1 0"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6cfgab2}; mkdir -p $O
VAR=${VAR:?set VAR}; VALS=${VALS:?set VALS}; CONFIG=${CONFIG:?set CONFIG}
for r in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python scripts/bench_configs.py --config $CONFIG --steps 6 --warmup 3 > $O/${v}_$r.log 2>&1 || { tail -20 $O/${v}_$r.log; exit 1; }
    echo "$VAR=$v $(tail -1 $O/${v}_$r.log | grep -o '"ms_per_round": [0-9.]*\|"device_allocs": [0-9]*' | tr '\n' ' ')"
  done
done

# device allocations inside the timed rounds (bench_configs.py device_allocs)
# with the side lane on / off, the headline bench with the lane
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6allocs}; mkdir -p $O
for v in 1 0; do
  COMMEFF_CONV_LANE=$v timeout -k 10 300 python scripts/bench_configs.py --config imagenet_local_topk --steps 6 --warmup ${WU:-2} > $O/img_$v.log 2>&1 || { tail -20 $O/img_$v.log; exit 1; }
  echo "lane=$v $(tail -1 $O/img_$v.log | grep -o '"ms_per_round": [0-9.]*\|"device_allocs": [0-9]*\|"host_ms_per_round": [0-9.]*' | tr '\n' ' ')"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
tail -1 $O/b.log | cut -c1-200

# GPT-2 round: host cProfile of the timed rounds + host/device sync report
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4l}
mkdir -p $O
COMMEFF_PROFILE_ROUNDS=$O/hp_rounds.txt timeout -k 10 300 python scripts/bench_configs.py --config gpt2_sketch --steps 30 --warmup 5 > $O/hp.log 2>&1 || { tail -20 $O/hp.log; exit 1; }
tail -1 $O/hp.log | cut -c1-200
head -75 $O/hp_rounds.txt
COMMEFF_SYNC_DEBUG=1 timeout -k 10 300 python scripts/bench_configs.py --config gpt2_sketch --steps 4 --warmup 3 > $O/sync.log 2>&1 || { tail -20 $O/sync.log; exit 1; }
grep SYNC $O/sync.log | sort | uniq -c | sort -rn | head -20

# ImageNet ResNet-101 local top-k: bench + kernel profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5inprof}
mkdir -p $O
timeout -k 10 400 python scripts/bench_configs.py --config imagenet_local_topk --steps 5 --warmup 2 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/prof -o run -- python scripts/bench_configs.py --config imagenet_local_topk --steps 3 --warmup 1 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python scripts/dev/rocpd_top.py $O/prof/run_results.db 4 45 > $O/top.txt && head -50 $O/top.txt

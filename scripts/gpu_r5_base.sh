# round-5 baseline: driver-shaped bench + per-layer conv timing (native vs MIOpen vs plain GEMM)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5base}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20_5_$r.log 2>&1 || { tail -20 $O/b20_5_$r.log; exit 1; }
  tail -1 $O/b20_5_$r.log | cut -c1-200
done
timeout -k 10 300 python scripts/bench_conv.py 500 > $O/conv500.log 2>&1 || { tail -20 $O/conv500.log; exit 1; }
cat $O/conv500.log
timeout -k 10 300 python scripts/bench_conv.py 2000 > $O/conv2000.log 2>&1 || { tail -20 $O/conv2000.log; exit 1; }
cat $O/conv2000.log

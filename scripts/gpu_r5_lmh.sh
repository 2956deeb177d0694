cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5lmh; mkdir -p $O
for r in 1 2; do
timeout -k 10 300 python scripts/bench_configs.py --config gpt2_sketch --steps 20 --warmup 3 > $O/blas$r.log 2>&1 || { tail -20 $O/blas$r.log; exit 1; }
tail -1 $O/blas$r.log | cut -c1-160
COMMEFF_LM_HEAD=native timeout -k 10 300 python scripts/bench_configs.py --config gpt2_sketch --steps 20 --warmup 3 > $O/nat$r.log 2>&1 || { tail -20 $O/nat$r.log; exit 1; }
tail -1 $O/nat$r.log | cut -c1-160
done

cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5g2tr2; mkdir -p $O
for r in 1 2; do
timeout -k 10 400 python scripts/bench_configs.py --config gpt2_sketch --steps 20 --warmup 3 > $O/b$r.log 2>&1 || { tail -20 $O/b$r.log; exit 1; }
tail -1 $O/b$r.log | cut -c1-200
done
COMMEFF_TORCH_PROFILE=/tmp/g2tr timeout -k 10 400 python scripts/bench_configs.py --config gpt2_sketch --steps 6 --warmup 3 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
python scripts/dev/trace_copies.py /tmp/g2tr/trace.json "Memcpy HtoD|copyBuffer|Memcpy DtoD|Memset" > $O/copies.txt 2>&1; head -30 $O/copies.txt

# GPT-2 round: quick bench x2 + driver tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4g2q}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_drivers.py tests/test_engine.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 0 1; do
  timeout -k 10 400 python scripts/bench_configs.py --config gpt2_sketch --steps 30 --warmup 5 > $O/g$r.log 2>&1 || { tail -20 $O/g$r.log; exit 1; }
  echo "gpt2 $r: $(tail -1 $O/g$r.log | cut -c1-260)"
done

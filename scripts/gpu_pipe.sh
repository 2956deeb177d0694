# persistent pipelined conv kernel with the DB/interleaved inner loop vs the halo kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4p}
mkdir -p $O
COMMEFF_CONV_PIPE=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv.py -k "fwd or dgrad or pool or residual or unit or accurate" > $O/pipe_tests.log 2>&1 || { echo PIPE_TESTS_FAILED; tail -30 $O/pipe_tests.log; exit 1; }
tail -1 $O/pipe_tests.log
for pp in 1 0; do
  COMMEFF_CONV_PIPE=$pp timeout -k 10 200 python scripts/conv_ablate.py > $O/layers_pipe$pp.log 2>&1 || { tail -5 $O/layers_pipe$pp.log; exit 1; }
  echo "pipe=$pp"; grep '^{' $O/layers_pipe$pp.log
done
for pp in 1 0; do
  COMMEFF_CONV_PIPE=$pp timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b_pipe$pp.log 2>&1 || { tail -20 $O/b_pipe$pp.log; exit 1; }
  echo "bench pipe=$pp $(tail -1 $O/b_pipe$pp.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["weights_checksum"])')"
done

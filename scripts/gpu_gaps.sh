# idle-gap analysis of the 1-GPU bench round (taped / eager, host-read staging
# kernel / runtime blit), then the staging and tape tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4h}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_hostcopy.py tests/test_conv.py -k "hostcopy or host_read or pinned or deferred or wgrad" > $O/hostcopy_tests.log 2>&1 || { echo HOSTCOPY_FAILED; tail -30 $O/hostcopy_tests.log; exit 1; }
tail -1 $O/hostcopy_tests.log
for v in ${VARIANTS:-tape notape tape_blit tape_nodefer}; do
  case $v in
    tape) E="" ;;
    notape) E="COMMEFF_TAPE=0" ;;
    tape_blit) E="COMMEFF_H2D=blit" ;;
    notape_blit) E="COMMEFF_TAPE=0 COMMEFF_H2D=blit" ;;
    tape_nodefer) E="COMMEFF_WGRAD_DEFER=0" ;;
  esac
  env $E timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b_$v.log 2>&1 || { tail -20 $O/b_$v.log; exit 1; }
  echo "$v $(tail -1 $O/b_$v.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["host_enqueue_ms_per_step"], r["config"]["round_tape"])')"
done
for v in ${TRACE_VARIANTS:-tape}; do
  case $v in
    tape) export COMMEFF_H2D=kernel COMMEFF_TAPE=1 ;;
    notape) export COMMEFF_H2D=kernel COMMEFF_TAPE=0 ;;
    tape_blit) export COMMEFF_H2D=blit COMMEFF_TAPE=1 ;;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/rp_$v -o bench -- python3 bench.py --steps 60 --warmup 20 > $O/rp_$v.log 2>&1 || exit 1
  python scripts/round_kernels.py $O/rp_$v/bench_kernel_trace.csv --marker cs_region_encode --rounds 30 --gaps 8 --top 60 > $O/rk_$v.txt 2>&1
  echo "== $v"; head -12 $O/rk_$v.txt
  rm -f $O/rp_$v/bench_kernel_trace.csv
done
unset COMMEFF_H2D COMMEFF_TAPE
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_tape.py > $O/tape_tests.log 2>&1 || { echo TAPE_TESTS_FAILED; tail -30 $O/tape_tests.log; exit 1; }
tail -2 $O/tape_tests.log
if [ -z "$SKIP_ABLATE" ]; then
for ab in 0 1 2 4 3 7; do
  COMMEFF_CONV_ABLATE=$ab timeout -k 10 200 python scripts/conv_ablate.py > $O/ablate_$ab.log 2>&1 || { tail -5 $O/ablate_$ab.log; exit 1; }
  grep '^{' $O/ablate_$ab.log
done
fi

# Ad-hoc GPU session: optional pytest selection then bench_configs runs.
#   TESTS="tests/test_conv.py -k native"  CONFIGS="imagenet_local_topk cifar100_fedavg"
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > gpurun_out/step_tests.log 2>&1
  rc=$?; tail -15 gpurun_out/step_tests.log; echo "tests rc=$rc"
  [ $rc -ne 0 ] && exit $rc
fi
for spec in $CONFIGS; do
  c=${spec%%:*}; extra=""
  if [ "$spec" != "$c" ]; then extra="${spec#*:}"; extra=${extra//=/ }; extra=${extra//,/ }; fi
  timeout -k 10 600 python scripts/bench_configs.py --config $c --steps ${STEPS:-5} --warmup 3 -- $extra > gpurun_out/step_$c.log 2>&1
  rc=$?; grep '"config"' gpurun_out/step_$c.log || tail -20 gpurun_out/step_$c.log; echo "$spec rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
[ -n "$BENCH" ] && { timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/step_bench.log 2>&1; rc=$?; tail -1 gpurun_out/step_bench.log; echo "bench rc=$rc"; }
exit 0

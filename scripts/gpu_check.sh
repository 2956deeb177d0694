#!/bin/bash
# One gpurun session: GPU tests, smoke, bench (+ optional rocprofv3 stats).
# Each GPU step has its own time limit; a fault-type exit (abort, segfault,
# timeout) stops the script so nothing else touches the GPU after it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-"build tests smoke bench"}

fault() {  # exit codes that mean the GPU step crashed or hung
  case "$1" in 124|134|137|139) return 0 ;; *) return 1 ;; esac
}

run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if fault $rc; then echo "FAULT in $name, stopping"; exit $rc; fi
  return 0
}

for s in $STEPS; do
  case $s in
    build) run build 300 python -m commefficient_amd.build ;;
    tests) run pytest_gpu 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps ${BENCH_STEPS:-30} --warmup 5 ;;
    benchprof) run bench_prof 600 python bench.py --steps 20 --warmup 5 --profile ;;
    codec) run codec 600 python scripts/bench_codec.py ;;
    conv) run conv 600 python scripts/bench_conv.py ;;
    convtest) run pytest_conv 600 python -m pytest tests/test_conv.py -x -q -m gpu ;;
    configs) for c in ${CONFIGS:-cifar100_fedavg imagenet_local_topk gpt2_sketch}; do
               run cfg_$c 900 python scripts/bench_configs.py --config $c; done ;;
    rocprof) run rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o bench \
               --output-format csv -- python3 bench.py --steps 10 --warmup 3 ;;
    *) echo "unknown step $s" ;;
  esac
done
echo ALL_DONE

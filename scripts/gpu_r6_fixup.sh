# FixupResNet9 native FedAvg: unit + round tests, then native vs vmap round time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6fixup}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests/test_fedavg_native.py -k "affine or fixup or resnet9 or supported or native_round" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
: > $O/configs.jsonl
for e in native vmap; do
  timeout -k 10 400 python scripts/bench_configs.py --config cifar10_resnet9_fedavg_local --steps 4 --warmup 2 -- --model FixupResNet9 --fedavg_engine $e > $O/$e.log 2>&1 || { tail -20 $O/$e.log; exit 1; }
  tail -1 $O/$e.log >> $O/configs.jsonl
  echo "$e: $(tail -1 $O/$e.log | cut -c1-200)"
done
for e in native vmap; do
  timeout -k 10 400 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 4 --warmup 2 -- --model FixupResNet18 --fedavg_engine $e > $O/r18_$e.log 2>&1 || { tail -20 $O/r18_$e.log; exit 1; }
  tail -1 $O/r18_$e.log >> $O/configs.jsonl
  echo "r18 $e: $(tail -1 $O/r18_$e.log | cut -c1-200)"
done

# ResNet-9 FedAvg: native G-client program tests, native vs vmap round time, native trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6fa9}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_fedavg_native.py tests/test_fedavg_batched.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
c=cifar10_resnet9_fedavg_local
: > $O/configs.jsonl
for e in native vmap native; do
  timeout -k 10 400 python scripts/bench_configs.py --config $c --steps 6 --warmup 2 -- --fedavg_engine $e > $O/$c.$e.log 2>&1 || { tail -20 $O/$c.$e.log; exit 1; }
  tail -1 $O/$c.$e.log >> $O/configs.jsonl
  echo "$e: $(tail -1 $O/$c.$e.log | cut -c1-260)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 scripts/bench_configs.py --config $c --steps 3 --warmup 2 -- --fedavg_engine native > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --tail-ms ${TAILMS:-200} --rounds 2 --top 60 > $O/rk.txt 2>&1
rm -f $O/rp/tr_kernel_trace.csv
head -50 $O/rk.txt

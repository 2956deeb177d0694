# batched FedAvg with the captured local step: equivalence tests + A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4fag}
mkdir -p $O
COMMEFF_FEDAVG_GRAPH=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_fedavg_batched.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for m in 1 0; do
  COMMEFF_FEDAVG_GRAPH=$m timeout -k 10 400 python scripts/bench_configs.py --config cifar100_fedavg_local --steps 4 --warmup 2 > $O/fa_$m.log 2>&1 || { tail -20 $O/fa_$m.log; exit 1; }
  echo "graph=$m: $(tail -1 $O/fa_$m.log | cut -c1-260)"
done

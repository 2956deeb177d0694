# full GPU suite, then the ImageNet config (2 runs) and its round trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6img}; mkdir -p $O
if [ -z "${NOTESTS:-}" ]; then
  timeout -k 10 1000 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/ ${TESTS:-} > $O/tests.log 2>&1
  rc=$?
  tail -8 $O/tests.log
  [ $rc -eq 0 ] || { echo "TESTS FAILED rc=$rc"; exit 1; }
fi
c=${CONFIG:-imagenet_local_topk}
: > $O/configs.jsonl
for r in 1 2; do
  timeout -k 10 400 python scripts/bench_configs.py --config $c --steps 8 --warmup 3 > $O/$c.$r.log 2>&1 || { tail -20 $O/$c.$r.log; exit 1; }
  tail -1 $O/$c.$r.log >> $O/configs.jsonl
  echo "$(tail -1 $O/$c.$r.log | cut -c1-330)"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 scripts/bench_configs.py --config $c --steps 4 --warmup 2 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --tail-ms ${TAILMS:-150} --rounds 3 --top 70 > $O/rk.txt 2>&1
rm -f $O/rp/tr_kernel_trace.csv
head -30 $O/rk.txt

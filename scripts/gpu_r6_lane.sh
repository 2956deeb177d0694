# side lane for the conv weight gradients (ops/lanes.py): tape tests, the
# driver-shaped bench alternating COMMEFF_CONV_LANE=1/0, one traced round
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6lane}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_tape.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 1 0; do
    COMMEFF_CONV_LANE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_${v}_${r}.log 2>&1 || { tail -20 $O/b_${v}_${r}.log; exit 1; }
    python -c "import json; r=json.loads(open('$O/b_${v}_${r}.log').read().strip().splitlines()[-1]); print('lane=$v bench', r['value'], r['ms_per_step'])"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o tr -- python3 bench.py --steps 20 --warmup 5 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/round_kernels.py $O/rp/tr_kernel_trace.csv --marker augment_kernel --rounds 12 --sequence --top 60 > $O/seq.txt 2>&1
rm -f $O/rp/tr_kernel_trace.csv
grep "^# rounds" $O/seq.txt

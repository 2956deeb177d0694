# A/B of two builds: abtest/_C_base.so (COMMEFF_LIB) vs the tree's _C.so -- tests on the new
# build, then a micro-benchmark and the driver-shaped bench alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6lib}; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $TESTS > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export COMMEFF_LIB=$PWD/abtest/_C_base.so; else unset COMMEFF_LIB; fi
    if [ -n "${MICRO:-}" ]; then
      timeout -k 10 200 python $MICRO > $O/micro_${v}_$r.log 2>&1 || { tail -20 $O/micro_${v}_$r.log; exit 1; }
      echo "$v micro: $(grep '^{' $O/micro_${v}_$r.log | cut -c1-400)"
    fi
    i=0
    IFS=';' read -ra BL <<< "${BARGS_LIST:- }"
    for ba in "${BL[@]}"; do
      i=$((i + 1))
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 $ba > $O/b_${v}_${r}_$i.log 2>&1 || { tail -20 $O/b_${v}_${r}_$i.log; exit 1; }
      python -c "import json; r=json.loads(open('$O/b_${v}_${r}_$i.log').read().strip().splitlines()[-1]); print('$v bench [$ba]', r['value'], r['ms_per_step'])"
    done
  done
done

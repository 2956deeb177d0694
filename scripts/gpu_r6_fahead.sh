# fused FedAvg classifier: tests, A/B on both FedAvg configs, kernel list of a ResNet-9 FedAvg round
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6fahead}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_fedavg_native.py tests/test_fedavg_batched.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in ${CONFIGS:-cifar10_resnet9_fedavg_local cifar100_fedavg_local}; do
  for r in 1 2; do
    for v in ${VALS:-1 0}; do
      env ${VAR:-COMMEFF_FA_HEAD}=$v timeout -k 10 300 python scripts/bench_configs.py --config $c --steps 6 --warmup 2 > $O/${c}_${v}_$r.log 2>&1 || { tail -20 $O/${c}_${v}_$r.log; exit 1; }
      python -c "import json; r=json.loads(open('$O/${c}_${v}_$r.log').read().strip().splitlines()[-1]); print('$c ${VAR:-COMMEFF_FA_HEAD}=$v', r['value'], r['ms_per_round'])"
    done
  done
done
rm -rf $O/rp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rp -o tr -- python3 scripts/bench_configs.py --config cifar10_resnet9_fedavg_local --steps 3 --warmup 2 > $O/rp.log 2>&1 || { tail -20 $O/rp.log; exit 1; }
python scripts/dev/rocpd_top.py $O/rp/tr_results.db 5 40 > $O/top.txt
grep -i "cijk\|fa_linear\|ce_fwd\|gemm_tn" $O/top.txt | cut -c1-150

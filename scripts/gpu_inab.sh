# ImageNet round A/B: native weight-gradient TN GEMMs vs hipBLASLt (alternating)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4inab}
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm.py -k "tn" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 0 1; do for m in 1 0; do
  COMMEFF_WGRAD_TN=$m timeout -k 10 400 python scripts/bench_configs.py --config imagenet_local_topk --steps 8 --warmup 2 > $O/in_${m}_$r.log 2>&1 || { tail -20 $O/in_${m}_$r.log; exit 1; }
  echo "tn=$m run $r: $(tail -1 $O/in_${m}_$r.log | cut -c1-200)"
done; done

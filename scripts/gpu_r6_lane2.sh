# side lane for every sunk conv weight gradient: the GPU tests that run the
# conv backward paths, then the ImageNet-shaped configs with the lane on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6lane2}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_tape.py tests/test_grouped.py tests/test_bn_epi.py tests/test_engine.py tests/test_fixup.py tests/test_determinism.py tests/test_im2col.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in imagenet_local_topk imagenet_fixup50_uncompressed; do
  for v in 1 0; do
    COMMEFF_CONV_LANE=$v timeout -k 10 300 python scripts/bench_configs.py --config $c --steps 6 --warmup 2 > $O/${c}_$v.log 2>&1 || { tail -20 $O/${c}_$v.log; exit 1; }
    echo "lane=$v $(tail -1 $O/${c}_$v.log | cut -c1-150)"
  done
done

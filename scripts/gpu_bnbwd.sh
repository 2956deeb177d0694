# BN backward partial with 4 pixels per step: BN tests, BN micro-benchmark, ImageNet round
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4bnb}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_conv.py tests/test_bn_epi.py tests/test_grouped.py tests/test_engine.py -k "bn or ghost or batchnorm or grouped" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python scripts/bench_bn.py > $O/bn.log 2>&1 || { tail -20 $O/bn.log; exit 1; }
grep -v amdgpu.ids $O/bn.log
timeout -k 10 400 python scripts/bench_configs.py --config imagenet_local_topk --steps 8 --warmup 2 > $O/in.log 2>&1 || { tail -20 $O/in.log; exit 1; }
echo "imagenet: $(tail -1 $O/in.log | cut -c1-200)"

# streamed conv kernel: numerics (conv GPU tests) + per-layer timing vs the per-tile halo kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5conv}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv.py > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python scripts/bench_conv.py 500 > $O/conv500_stream.log 2>&1 || { tail -20 $O/conv500_stream.log; exit 1; }
COMMEFF_CONV_STREAM=0 timeout -k 10 300 python scripts/bench_conv.py 500 > $O/conv500_halo.log 2>&1 || exit 1
python - <<'PY'
import json
O = "gpurun_out/" + __import__("os").environ.get("TAG", "r5conv")
for tag in ("stream", "halo"):
    for l in open(f"{O}/conv500_{tag}.log"):
        if l.startswith("{\"layer"):
            r = json.loads(l)
            print(tag, r["layer"], "fwd", r["fwd_native_us"], r["fwd_native_tflops"], "dgrad", r["dgrad_native_us"], r["dgrad_native_tflops"])
PY

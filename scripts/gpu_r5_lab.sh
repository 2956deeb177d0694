# streamed conv: numerics + timing variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5lab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv.py > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit $rc
run() { timeout -k 10 120 env "$@" python scripts/dev/stream_lab.py >> $O/lab.jsonl 2>>$O/lab.err || { tail -5 $O/lab.err; exit 1; }; }
run COMMEFF_CONV_STREAM=0 TAG=halo
run TAG=stream
run TAG=narrow0 COMMEFF_STREAM_NARROW=0
run TAG=narrow1 COMMEFF_STREAM_NARROW=1
run TAG=ab8 COMMEFF_STREAM_ABLATE=8
run TAG=ab15 COMMEFF_STREAM_ABLATE=15
cat $O/lab.jsonl

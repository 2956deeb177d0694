cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5g2chk; mkdir -p $O
timeout -k 10 300 python scripts/dev/gpt2_native_vs_stock.py > $O/cmp.log 2>&1; rc=$?
tail -30 $O/cmp.log; exit $rc

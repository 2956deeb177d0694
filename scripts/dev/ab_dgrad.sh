cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
for v in -1 -1; do
  echo "small=$v"; COMMEFF_TN_SMALL_AB=$v timeout -k 10 120 python3 scripts/bench_gemm_tn.py || exit 1
done

# halo conv forward ablations (timing only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4n}
mkdir -p $O
for ab in ${ABLATE:-0 8 7 15}; do
  COMMEFF_CONV_ABLATE=$ab timeout -k 10 200 python scripts/conv_ablate.py > $O/ablate_$ab.log 2>&1 || { tail -5 $O/ablate_$ab.log; exit 1; }
  grep '^{' $O/ablate_$ab.log
done

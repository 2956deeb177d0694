# A/B sweep of the conv dispatch knobs on the 1-GPU bench (200 timed after 50)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4z}
mkdir -p $O
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b_$tag.log 2>&1 || { tail -5 $O/b_$tag.log; return 1; }
  echo "$tag $(tail -1 $O/b_$tag.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
}
run base0 X=0 || exit 1
run tbm128 COMMEFF_CONV_HALO_TBM=128 || exit 1
run nosplit COMMEFF_CONV_SPLIT=0 || exit 1
run wg3 COMMEFF_WGRAD_HALO_STAGES=3 || exit 1
run wideil COMMEFF_WGRAD_WIDE_IL=1 || exit 1
run nohalo64 COMMEFF_CONV_HALO64=0 || exit 1
run wide COMMEFF_CONV_WIDE=1 || exit 1
run base1 X=1 || exit 1

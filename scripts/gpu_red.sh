# narrow-row wgrad split reduction: conv tests + same-box A/B (200 timed after 50)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4red}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv.py -k "wgrad" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $O/b_$tag.log 2>&1 || { tail -5 $O/b_$tag.log; return 1; }
  echo "$tag $(tail -1 $O/b_$tag.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r.get("weights_checksum", ""))')"
}
run n1a COMMEFF_WGRAD_RED_NARROW=1 || exit 1
run n0a COMMEFF_WGRAD_RED_NARROW=0 || exit 1
run n1b COMMEFF_WGRAD_RED_NARROW=1 || exit 1
run n0b COMMEFF_WGRAD_RED_NARROW=0 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o bench -- python3 bench.py --steps 20 --warmup 5 > $O/rp.log 2>&1 || exit 1
python scripts/round_kernels.py $O/rp/bench_kernel_trace.csv --marker cs_region_encode --rounds 8 --top 30 > $O/rk.txt 2>&1
head -30 $O/rk.txt
rm -f $O/rp/bench_kernel_trace.csv

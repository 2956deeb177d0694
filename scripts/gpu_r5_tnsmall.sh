cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r5tns; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm.py tests/test_im2col.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python scripts/bench_configs.py --config imagenet_local_topk --steps 5 --warmup 2 > $O/in.log 2>&1 || { tail -30 $O/in.log; exit 1; }
tail -1 $O/in.log
timeout -k 10 500 rocprofv3 --kernel-trace -d $O/prof -o run -- python scripts/bench_configs.py --config imagenet_local_topk --steps 3 --warmup 1 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python scripts/dev/rocpd_top.py $O/prof/run_results.db 4 30 > $O/top.txt && head -32 $O/top.txt

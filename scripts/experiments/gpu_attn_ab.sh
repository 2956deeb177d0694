# long attention kernels: tests + micro-benchmark A/B (transposed vs image forms)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_transformer.py -x -q -m gpu -k "attention or fused" --timeout 120 --timeout-method thread > gpurun_out/attn_ab_tests.log 2>&1 || { tail -40 gpurun_out/attn_ab_tests.log; exit 1; }
tail -1 gpurun_out/attn_ab_tests.log
timeout -k 10 120 python3 scripts/bench_attention.py --p 0.1 || exit 1
COMMEFF_ATTN_DKDV_S=0 timeout -k 10 120 python3 scripts/bench_attention.py --p 0.1 || exit 1
COMMEFF_ATTN_DQ_T=0 timeout -k 10 120 python3 scripts/bench_attention.py --p 0.1 || exit 1
COMMEFF_ATTN_FWD_T=0 COMMEFF_ATTN_DQ_T=0 timeout -k 10 120 python3 scripts/bench_attention.py --p 0.1 || exit 1

set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transformer.py -x -q -m gpu -k "gemm_tn or attention or native" --timeout 250 --timeout-method thread > gpurun_out/r3_pytest_d.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r3_pytest_d.log; exit 1; }
tail -2 gpurun_out/r3_pytest_d.log
timeout -k 10 200 python -u scripts/dev/bench_gpt2_wgrad.py 2>&1 | grep -v amdgpu
timeout -k 10 300 python -u scripts/bench_configs.py --config gpt2_sketch > gpurun_out/r3_gpt2_d.log 2>&1
tail -1 gpurun_out/r3_gpt2_d.log
COMMEFF_WGRAD_GEMM=blas timeout -k 10 300 python -u scripts/bench_configs.py --config gpt2_sketch > gpurun_out/r3_gpt2_d_blas.log 2>&1
tail -1 gpurun_out/r3_gpt2_d_blas.log

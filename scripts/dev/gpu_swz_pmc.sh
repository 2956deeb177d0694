# LDS conflict counters of the conv kernels, halo swizzle on / off
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_swz_on -o run -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/pmc_swz_on.log 2>&1 || exit 1
COMMEFF_HALO_SWIZZLE=0 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_swz_off -o run -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/pmc_swz_off.log 2>&1 || exit 1
echo OK

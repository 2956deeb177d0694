# attention micro-benchmark + one PMC pass over its kernels
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/bench_attention.py --p 0.1
timeout -k 10 120 python3 scripts/bench_attention.py --p 0.0
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d gpurun_out/pmc_attn -o run -- python3 scripts/bench_attention.py --p 0.1 > gpurun_out/pmc_attn.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/pmc_attn2 -o run -- python3 scripts/bench_attention.py --p 0.1 > gpurun_out/pmc_attn2.log 2>&1
echo DONE

#!/bin/bash
# PMC counters of the native conv kernels (two passes; --pmc only with
# --kernel-trace-free collection as the pool requires).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
V=${VARIANT:-glds}
if [ "$V" = regs ]; then export COMMEFF_CONV_FWD=regs; fi
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT \
  --output-format csv -d gpurun_out/pmc/$V.sq -o run -- python3 scripts/prof_conv.py "$@" > gpurun_out/pmc/$V.sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
  --output-format csv -d gpurun_out/pmc/$V.tcc -o run -- python3 scripts/prof_conv.py "$@" > gpurun_out/pmc/$V.tcc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES \
  --output-format csv -d gpurun_out/pmc/$V.mfma -o run -- python3 scripts/prof_conv.py "$@" > gpurun_out/pmc/$V.mfma.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/$V.kt -o run -- python3 scripts/prof_conv.py "$@" > gpurun_out/pmc/$V.kt.log 2>&1

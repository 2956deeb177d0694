#!/bin/bash
# usage: pmc_generic.sh NAME script.py [args...]  -> gpurun_out/pmc/NAME.{sq,tcc,kt}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
N=$1; shift
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT \
  --output-format csv -d gpurun_out/pmc/$N.sq -o run -- python3 "$@" > gpurun_out/pmc/$N.sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
  --output-format csv -d gpurun_out/pmc/$N.tcc -o run -- python3 "$@" > gpurun_out/pmc/$N.tcc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/$N.kt -o run -- python3 "$@" > gpurun_out/pmc/$N.kt.log 2>&1

#!/bin/bash
# Hardware counters per kernel of a program, four rocprofv3 passes (each pass
# stays inside the gfx950 per-block slot limits: <= 8 SQ, <= 4 TCC, <= 2 GRBM;
# --pmc is combined only with --kernel-trace), then scripts/pmc_summary.py.
#   TAG=headline scripts/pmc_bench.sh bench.py --steps 4 --warmup 2
#   TAG=gpt2 scripts/pmc_bench.sh scripts/bench_configs.py --config gpt2_sketch --steps 2 --warmup 1
# -> gpurun_out/pmc_$TAG/{p1..p4}/ and gpurun_out/pmc_$TAG/summary.txt
# ONLY="1 3" runs a subset of the passes; SUMMARY_ARGS="--marker enc_p1 --rounds 4"
# restricts the summary to the last 4 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
  "FETCH_SIZE GRBM_GUI_ACTIVE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"
)
i=0
DIRS=""
for ctrs in "${PASSES[@]}"; do
  i=$((i + 1))
  case " ${ONLY:-1 2 3 4} " in *" $i "*) ;; *) continue;; esac
  DIRS="$DIRS $OUT/p$i"
  echo "=== pass p$i: $ctrs"
  timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/p$i -o run \
    -- python3 "$@" > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; exit $rc; fi
done
python3 scripts/pmc_summary.py $DIRS --top 40 ${SUMMARY_ARGS:-} > $OUT/summary.txt
rc=$?
# raw per-dispatch CSVs are large (gpurun copies back <= 64 MiB): kept only on request
[ -n "${KEEP_RAW:-}" ] || rm -rf $DIRS
cat $OUT/summary.txt
exit $rc

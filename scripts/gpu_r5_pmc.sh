# PMC counters of the conv kernels on the ResNet-9 layer shapes (stream vs halo)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r5pmc}
mkdir -p $O
for V in stream halo; do
  if [ $V = halo ]; then export COMMEFF_CONV_STREAM=0; else unset COMMEFF_CONV_STREAM; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS \
    --output-format csv -d $O/$V.sq -o run -- python3 scripts/dev/stream_lab.py > $O/$V.sq.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU \
    --output-format csv -d $O/$V.mf -o run -- python3 scripts/dev/stream_lab.py > $O/$V.mf.log 2>&1 || exit 1
done
python3 scripts/dev/pmc_sum.py $O/stream.sq $O/stream.mf $O/halo.sq $O/halo.mf > $O/summary.txt 2>&1
cat $O/summary.txt

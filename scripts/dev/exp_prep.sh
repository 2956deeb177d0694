#!/bin/bash
# input-conv forward: tiles per wave sweep (kernel stats under rocprofv3)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in 4 1 2 8; do
  COMMEFF_PREP_TPW=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prep_$t -o s --output-format csv -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prep_$t.log 2>&1 || exit 1
  echo "tpw=$t"; grep -h "prep_fwd_kernel\|prep_wgrad_kernel" gpurun_out/prep_$t/s_kernel_stats.csv | cut -d, -f1-5
done

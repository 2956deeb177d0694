set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
MODES=${MODES:-"native hf"}
for mode in $MODES; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$mode -o tr -- python3 scripts/bench_configs.py --config gpt2_sketch --steps 4 --warmup 2 -- --transformer $mode > gpurun_out/prof_$mode.log 2>&1
done

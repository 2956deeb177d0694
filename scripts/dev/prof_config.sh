set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=${CFG:-imagenet_local_topk}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$CFG -o tr -- python3 scripts/bench_configs.py --config $CFG --steps 3 --warmup 2 > gpurun_out/prof_$CFG.log 2>&1

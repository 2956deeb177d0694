set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_head -o tr -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_head.log 2>&1

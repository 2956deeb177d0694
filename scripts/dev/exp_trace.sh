#!/bin/bash
# kernel trace of a few headline rounds (optionally with env overrides passed in $EXTRA_ENV)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/rocprof.log 2>&1
rc=$?
tail -n 2 gpurun_out/rocprof.log
exit $rc

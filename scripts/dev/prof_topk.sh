cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_tk -o run -- python3 scripts/bench_codec.py resnet9 > gpurun_out/rp_tk.log 2>&1; echo rc=$?

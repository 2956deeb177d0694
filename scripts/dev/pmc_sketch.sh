cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc
timeout -k 10 200 python scripts/bench_codec.py resnet9 > gpurun_out/codec.log 2>&1; echo codec rc=$?; tail -2 gpurun_out/codec.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/sk.kt -o run -- python3 scripts/prof_codec.py > gpurun_out/pmc/sk.kt.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc/sk.sq -o run -- python3 scripts/prof_codec.py > gpurun_out/pmc/sk.sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d gpurun_out/pmc/sk.tcc -o run -- python3 scripts/prof_codec.py > gpurun_out/pmc/sk.tcc.log 2>&1 || exit $?
echo done

# effective clock + MFMA busy per kernel: conv_lab alone and the headline bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6clk}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $O/lab -o run -- python3 scripts/dev/conv_lab.py > $O/lab.log 2>&1 || { tail -5 $O/lab.log; exit 1; }
python scripts/dev/pmc_clock.py $O/lab conv > $O/lab_clock.txt && cat $O/lab_clock.txt
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $O/bench -o run -- python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python scripts/dev/pmc_clock.py $O/bench > $O/bench_clock.txt && head -30 $O/bench_clock.txt
rm -f $O/*/*/*.csv $O/*/*.csv 2>/dev/null; true

# ImageNet + GPT-2: kernel splits and host profiles of the current tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4v}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/rp_in -o bench -- python3 scripts/bench_configs.py --config imagenet_local_topk --steps 4 --warmup 2 > $O/rp_in.log 2>&1 || { tail -5 $O/rp_in.log; exit 1; }
python scripts/round_kernels.py $O/rp_in/bench_kernel_trace.csv --marker write_kernel --rounds 3 --top 45 > $O/rk_in.txt 2>&1
head -48 $O/rk_in.txt
rm -f $O/rp_in/bench_kernel_trace.csv
COMMEFF_PROFILE_ROUNDS=$O/hp_gpt2.txt timeout -k 10 300 python scripts/bench_configs.py --config gpt2_sketch --steps 30 --warmup 5 > $O/hp_gpt2.log 2>&1 || exit 1
sed -n '/Ordered by: cumulative/,$p' $O/hp_gpt2.txt | head -75

# kernel trace of the ImageNet ResNet-101 local top-k round (per-round kernel table)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r3_imagenet}
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$TAG -o tr -- python3 scripts/bench_configs.py --config imagenet_local_topk --steps 4 --warmup 2 > gpurun_out/prof_$TAG.log 2>&1
python3 scripts/round_kernels.py $(find gpurun_out/prof_$TAG -name "*kernel_trace.csv" | head -1) --rounds 3 --top 70 > gpurun_out/${TAG}_round_kernels.txt
rm -rf gpurun_out/prof_$TAG
tail -1 gpurun_out/prof_$TAG.log
echo PROF_DONE

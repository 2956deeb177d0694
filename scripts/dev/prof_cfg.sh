# rocprofv3 per-round kernel split of the secondary configs
# (scripts/bench_configs.py): the trace is summarised on the box over the
# timed rounds and deleted (only the summaries travel back).
# CONFIGS="name[:extra flags]" entries, e.g. "gpt2_sketch:--encode=direct".
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_cfg
STEPS=${STEPS:-3}
for spec in ${CONFIGS:-imagenet_local_topk gpt2_sketch cifar100_fedavg}; do
  c=${spec%%:*}; extra=""; tag=$c
  if [ "$spec" != "$c" ]; then extra="${spec#*:}"; extra=${extra//=/ }; tag="${c}_$(echo ${spec#*:} | tr -c 'a-zA-Z0-9\n' '_')"; fi
  echo "=== $tag ($extra)"
  timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_$tag -o k --output-format csv -- python3 scripts/bench_configs.py --config $c --steps $STEPS --warmup 2 -- $extra > gpurun_out/prof_cfg/$tag.log 2>&1
  rc=$?; echo rc=$rc
  case $rc in 124|134|137|139) tail -20 gpurun_out/prof_cfg/$tag.log; exit $rc;; esac
  line=$(grep '"config"' gpurun_out/prof_cfg/$tag.log); echo "$line"
  ms=$(echo "$line" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_round'])")
  tail_ms=$(python3 -c "print($ms*$STEPS)")
  python3 scripts/round_kernels.py /tmp/prof_$tag/k_kernel_trace.csv --tail-ms $tail_ms --rounds $STEPS --top 60 > gpurun_out/prof_cfg/${tag}_round.txt
  head -30 gpurun_out/prof_cfg/${tag}_round.txt
  rm -rf /tmp/prof_$tag
done

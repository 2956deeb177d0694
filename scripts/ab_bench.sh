#!/bin/bash
# Same-box A/B of bench.py argument sets (box-to-box variance is ~4 %):
# alternates the variants ROUNDS times, one JSON line each into
# gpurun_out/${TAG}_ab.jsonl.
#   A="--wgrad-stream off" B="--wgrad-stream on" ROUNDS=3 bash scripts/ab_bench.sh
# AENV / BENV: environment assignments for a variant (AENV="COMMEFF_CONV_LANE=0")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-ab}
out=gpurun_out/${TAG}_ab.jsonl
: > "$out"
for i in $(seq "${ROUNDS:-3}"); do
  for v in A B; do
    envv=${v}ENV
    timeout -k 10 200 env ${!envv} python bench.py ${!v} > gpurun_out/${TAG}_ab_run.log 2>&1 || { tail -20 gpurun_out/${TAG}_ab_run.log; exit 1; }
    echo "{\"variant\": \"$v\", \"args\": \"${!envv} ${!v}\", \"result\": $(tail -1 gpurun_out/${TAG}_ab_run.log)}" >> "$out"
    python -c "import json,sys; r=json.loads(sys.argv[1]); print('$v', r['value'], r['ms_per_step'])" "$(tail -1 gpurun_out/${TAG}_ab_run.log)"
  done
done

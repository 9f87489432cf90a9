#!/bin/bash
# A/B of an environment switch on the training bench: for each value, one bench run.
# usage: VAR=RAFT_WGRAD_SPLIT VALUES="1 2 3" bash scripts/ab_env.sh [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for v in $VALUES; do
  env $VAR=$v timeout -k 10 300 python -u bench.py ${@:---steps 30 --warmup 5} > gpurun_out/ab/$VAR-$v.log 2>&1 || { echo "$VAR=$v failed"; tail -5 gpurun_out/ab/$VAR-$v.log; exit 1; }
  echo "$VAR=$v $(grep -o '"value": [0-9.]*' gpurun_out/ab/$VAR-$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/$VAR-$v.log)"
done

#!/bin/bash
for r in 1 2; do
bash scripts/gpu_step.sh \
 "150 r4ai_def$r.json python bench.py --steps 40" \
 "150 r4ai_lead3_$r.json env RAFT_MAX_LEAD=3 python bench.py --steps 40" \
 "150 r4ai_ws2_$r.json env RAFT_WGRAD_STREAMS=2 python bench.py --steps 40" \
 "150 r4ai_nohp$r.json env RAFT_HP_MAIN=0 python bench.py --steps 40" \
 "150 r4ai_lead1_$r.json env RAFT_MAX_LEAD=1 python bench.py --steps 40" || exit 1
done

#!/bin/bash
bash scripts/gpu_step.sh \
 "150 r4w_a1.json python bench.py --steps 40" \
 "150 r4w_gc1.json env RAFT_GC_FREEZE=1 python bench.py --steps 40" \
 "150 r4w_a2.json python bench.py --steps 40" \
 "150 r4w_gc2.json env RAFT_GC_FREEZE=1 python bench.py --steps 40" \
 "150 r4w_a3.json python bench.py --steps 40" \
 "150 r4w_gc3.json env RAFT_GC_FREEZE=1 python bench.py --steps 40"

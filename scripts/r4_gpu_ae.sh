#!/bin/bash
bash scripts/gpu_step.sh \
 "150 r4ae_steps40.log env RAFT_BENCH_STEP_TIMES=1 python bench.py --steps 40 --warmup 5" \
 "150 r4ae_steps20.log env RAFT_BENCH_STEP_TIMES=1 python bench.py --steps 20 --warmup 5" \
 "150 r4ae_steps20w15.log env RAFT_BENCH_STEP_TIMES=1 python bench.py --steps 20 --warmup 15"

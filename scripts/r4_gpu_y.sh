#!/bin/bash
bash scripts/gpu_step.sh \
 "150 r4y_a1.json python bench.py --steps 40" \
 "150 r4y_np1.json env RAFT_ENC_PREPACK=0 python bench.py --steps 40" \
 "150 r4y_fwd1.json env RAFT_ENC_PREPACK=fwd python bench.py --steps 40" \
 "150 r4y_same1.json env RAFT_ENC_PREPACK=same python bench.py --steps 40" \
 "150 r4y_np2.json env RAFT_ENC_PREPACK=0 python bench.py --steps 40" \
 "150 r4y_fwd2.json env RAFT_ENC_PREPACK=fwd python bench.py --steps 40" \
 "150 r4y_same2.json env RAFT_ENC_PREPACK=same python bench.py --steps 40" \
 "150 r4y_a2.json python bench.py --steps 40"

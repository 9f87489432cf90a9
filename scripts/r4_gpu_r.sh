#!/bin/bash
bash scripts/gpu_step.sh \
 "120 r4r_norm_default.log python scripts/bench_norm_bwd.py" \
 "120 r4r_norm_r128.log env RAFT_NORM_R=128 RAFT_NORM_PIX=128 python scripts/bench_norm_bwd.py" \
 "120 r4r_norm_r256.log env RAFT_NORM_R=256 RAFT_NORM_PIX=64 python scripts/bench_norm_bwd.py" \
 "120 r4r_norm_r32.log env RAFT_NORM_R=32 python scripts/bench_norm_bwd.py"

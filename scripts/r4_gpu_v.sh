#!/bin/bash
bash scripts/gpu_step.sh \
 "120 r4v_n2_2048.log python scripts/bench_conv6.py --only heads --cfgs 41" \
 "200 r4v_convs_2048.log python scripts/bench_convs.py" \
 "200 r4v_convs_512.log env RAFT_N2_BLOCKS=512 python scripts/bench_convs.py" \
 "200 r4v_convs_256.log env RAFT_N2_BLOCKS=256 python scripts/bench_convs.py" \
 "200 r4v_convs_1024.log env RAFT_N2_BLOCKS=1024 python scripts/bench_convs.py"

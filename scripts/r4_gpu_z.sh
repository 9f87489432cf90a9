#!/bin/bash
bash scripts/gpu_step.sh \
 "200 r4z_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_encoder_gpu.py -k prepack" \
 "150 r4z_a1.json python bench.py --steps 40" \
 "150 r4z_np1.json env RAFT_ENC_PREPACK=0 python bench.py --steps 40" \
 "150 r4z_same1.json env RAFT_ENC_PREPACK=same python bench.py --steps 40" \
 "150 r4z_a2.json python bench.py --steps 40" \
 "150 r4z_np2.json env RAFT_ENC_PREPACK=0 python bench.py --steps 40" \
 "150 r4z_same2.json env RAFT_ENC_PREPACK=same python bench.py --steps 40"

#!/bin/bash
bash scripts/gpu_step.sh \
 "300 r4x_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_train_graph.py tests/test_split_train_gpu.py" \
 "150 r4x_a1.json python bench.py --steps 40" \
 "150 r4x_np1.json env RAFT_ENC_PREPACK=0 python bench.py --steps 40" \
 "150 r4x_a2.json python bench.py --steps 40" \
 "150 r4x_np2.json env RAFT_ENC_PREPACK=0 python bench.py --steps 40" \
 "150 r4x_a3.json python bench.py --steps 40" \
 "150 r4x_np3.json env RAFT_ENC_PREPACK=0 python bench.py --steps 40" \
 "200 r4x_f1.json python bench.py --steps 20 --fp32" \
 "200 r4x_fn1.json env RAFT_ENC_PREPACK=0 python bench.py --steps 20 --fp32"

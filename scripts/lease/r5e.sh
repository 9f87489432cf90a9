#!/bin/bash
# round 5, lease e: three-plane fp32 encoder forward (split mode 2) -- golden gradients, encoder tests, fp32 bench
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
bash scripts/gpu_step.sh \
 "600 r5e_tests.log $T tests/test_golden_gpu.py tests/test_encoder_gpu.py tests/test_split_train_gpu.py" \
 "200 r5e_bench_fp32.json python bench.py --fp32" \
 "200 r5e_bench_fp32_old.json env RAFT_ENC_SPLIT3=0 python bench.py --fp32" \
 "200 r5e_bench.json python bench.py"

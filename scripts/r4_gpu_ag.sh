#!/bin/bash
bash scripts/gpu_step.sh \
 "400 r4ag_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_update_fused_gpu.py tests/test_golden_gpu.py tests/test_split_train_gpu.py" \
 "150 r4ag_c2_a1.json python bench.py --steps 40" \
 "200 r4ag_s_a1.json python bench.py --steps 20 --batch 6 --image_size 368 768" \
 "200 r4ag_1080_a1.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "150 r4ag_c2_a2.json python bench.py --steps 40" \
 "200 r4ag_s_a2.json python bench.py --steps 20 --batch 6 --image_size 368 768"

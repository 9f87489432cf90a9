#!/bin/bash
# round 5, lease aa: no per-iteration hidden-state copy in inference
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
I="python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "400 r5aa_tests.log $T tests/test_model_gpu.py tests/test_update_fused_gpu.py tests/test_fp16_gpu.py tests/test_golden_gpu.py" \
 "200 r5aa_1080.json $I" \
 "200 r5aa_1080_b.json $I" \
 "200 r5aa_sintel.json python bench.py --mode infer --image_size 440 1024 --iters 32 --batch 1 --steps 20 --warmup 3" \
 "200 r5aa_small.json python bench.py --mode infer --small --image_size 440 1024 --iters 32 --batch 1 --steps 20 --warmup 3" \
 "200 r5aa_bench.json python bench.py"

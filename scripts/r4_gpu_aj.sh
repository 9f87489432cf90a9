#!/bin/bash
bash scripts/gpu_step.sh \
 "300 r4aj_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_golden_gpu.py -k lookup\ or\ bf16\ or\ pyramid" \
 "200 r4aj_1080_new1.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "200 r4aj_1080_old1.json env RAFT_LOOKUP_ALL=0 python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "150 r4aj_c2_new1.json python bench.py --steps 40" \
 "150 r4aj_c2_old1.json env RAFT_LOOKUP_ALL=0 python bench.py --steps 40" \
 "200 r4aj_1080_new2.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "200 r4aj_1080_old2.json env RAFT_LOOKUP_ALL=0 python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "150 r4aj_c2_new2.json python bench.py --steps 40" \
 "150 r4aj_c2_old2.json env RAFT_LOOKUP_ALL=0 python bench.py --steps 40"

#!/bin/bash
# round 5, lease ai: 1x1 GEMM (conv_fwd7) on a 2-stage ring, three workgroups per CU
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5ai_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k 'full_size and (67 or 71)'" \
 "200 r5ai_convs.log python scripts/bench_convs.py --cfg 67,71" \
 "200 r5ai_ring3.json python bench.py" \
 "200 r5ai_ring2.json env RAFT_V7_RING2=1 python bench.py" \
 "200 r5ai_ring3b.json python bench.py" \
 "200 r5ai_ring2b.json env RAFT_V7_RING2=1 python bench.py" \
 "200 r5ai_1080_ring3.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "200 r5ai_1080_ring2.json env RAFT_V7_RING2=1 python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3"

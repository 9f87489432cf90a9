#!/bin/bash
bash scripts/gpu_step.sh \
 "400 r4ak_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_split_train_gpu.py tests/test_fp16_gpu.py tests/test_golden_gpu.py tests/test_model_gpu.py" \
 "200 r4ak_ros_new1.json python bench.py --mode infer --fp32 --image_size 440 1024 --iters 20 --batch 1 --steps 10 --warmup 3" \
 "200 r4ak_ros_old1.json env RAFT_LOOKUP_ALL=0 python bench.py --mode infer --fp32 --image_size 440 1024 --iters 20 --batch 1 --steps 10 --warmup 3" \
 "200 r4ak_f32_new1.json python bench.py --fp32 --steps 20" \
 "200 r4ak_f32_old1.json env RAFT_LOOKUP_ALL=0 python bench.py --fp32 --steps 20" \
 "200 r4ak_ros_new2.json python bench.py --mode infer --fp32 --image_size 440 1024 --iters 20 --batch 1 --steps 10 --warmup 3" \
 "200 r4ak_ros_old2.json env RAFT_LOOKUP_ALL=0 python bench.py --mode infer --fp32 --image_size 440 1024 --iters 20 --batch 1 --steps 10 --warmup 3"

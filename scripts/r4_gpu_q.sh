#!/bin/bash
bash scripts/gpu_step.sh \
 "300 r4q_tests.log python -u -m pytest tests/test_model_gpu.py tests/test_encoder_gpu.py -q --timeout 300 --timeout-method thread" \
 "200 r4q_bench_sintel_fp32.json python bench.py --fp32 --batch 6 --image_size 368 768 --steps 8 --warmup 3" \
 "200 r4q_bench_sintel.json python bench.py --batch 6 --image_size 368 768 --steps 20" \
 "200 r4q_bench_full.json python bench.py --batch 6 --image_size 440 1024 --steps 15" \
 "200 r4q_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "200 r4q_bench_kitti_dense.json python bench.py --batch 3 --image_size 376 1248 --steps 15" \
 "200 r4q_bench_infer_sintel.json python bench.py --mode infer --image_size 440 1024 --iters 32 --batch 1 --steps 20 --warmup 3" \
 "200 r4q_bench_ros_fp32.json python bench.py --mode infer --fp32 --image_size 440 1024 --iters 20 --batch 1 --steps 20 --warmup 3"

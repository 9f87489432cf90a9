#!/bin/bash
# The current GPU session plan (one gpurun call): steps run in order by scripts/gpu_step.sh,
# each "<timeout s> <log under gpurun_out/> <command>"; the first crash / time-out ends it.
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
bash scripts/gpu_step.sh \
 "600 r6f_tests.log $T tests/test_optim_gpu.py tests/test_encoder_gpu.py tests/test_golden_gpu.py tests/test_kernels_gpu.py tests/test_split_train_gpu.py tests/test_fp16_gpu.py tests/test_ddp_gpu.py" \
 "200 r6f_bench.json python bench.py" \
 "200 r6f_bench2.json python bench.py" \
 "200 r6f_bench_fp32.json python bench.py --fp32" \
 "200 r6f_bench_fp16.json python bench.py --amp_dtype fp16" \
 "200 r6f_b1_368x768.json python bench.py --batch 1 --image_size 368 768" \
 "200 r6f_b2_368x768.json python bench.py --batch 2 --image_size 368 768" \
 "200 r6f_b6_368x768.json python bench.py --batch 6 --image_size 368 768"

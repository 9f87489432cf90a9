#!/bin/bash
# round 5, lease n: corr volume v3 (BK 32, 4 WG/CU, swapped-operand epilogue); n2_apply branch-free
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5n_tests.log $T tests/test_kernels_gpu.py tests/test_conv_gpu.py -k corr_volume_v2_matches_generic\ or\ flow_head_conv2" \
 "300 r5n_bench_corr.log python scripts/bench_corr.py" \
 "200 r5n_bench_1080.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "200 r5n_bench.json python bench.py"

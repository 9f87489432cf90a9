#!/bin/bash
# round 5, lease c: new choose_fwd6 rule (128x64 two-workgroup tiles) -- numerics, then step benches
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash scripts/gpu_step.sh \
 "400 r5c_tests.log $T tests/test_conv_gpu.py tests/test_update_fused_gpu.py tests/test_golden_gpu.py tests/test_fp16_gpu.py tests/test_split_train_gpu.py" \
 "300 r5c_conv6_15.log python scripts/bench_conv6.py --cfgs 41,59,62,65 --only zr,q15,d_zr15,d_q15,heads,d_convc2" \
 "300 r5c_conv6_15_1080.log python scripts/bench_conv6.py --cfgs 41,59,62,65 --batch 1 --hw 135 240 --only zr,q15,d_zr15,d_q15" \
 "300 r5c_conv6_15_kitti.log python scripts/bench_conv6.py --cfgs 41,59,62,65 --batch 3 --hw 47 156 --only zr,q15,d_zr15,d_q15,zr51,d_zr51" \
 "200 r5c_bench.json python bench.py" \
 "200 r5c_bench2.json python bench.py" \
 "200 r5c_bench_1080.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "200 r5c_bench_sintel.json python bench.py --batch 6 --image_size 368 768" \
 "200 r5c_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15"

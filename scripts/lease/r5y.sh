#!/bin/bash
# round 5, lease y: n2_apply as pixel x slot waves; 4-stage weight ring for the 128x64 conv tiles (cfg 70)
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
I="python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "400 r5y_tests.log $T tests/test_conv_gpu.py tests/test_update_fused_gpu.py" \
 "120 r5y_n2.log python scripts/bench_n2_apply.py" \
 "300 r5y_conv6.log python scripts/bench_conv6.py --cfgs 62,70 --only conv,convc2,heads,d_conv,d_convc2,d_fh1,zr,q15,zr51,q51,d_zr15,d_zr51" \
 "300 r5y_conv6_1080.log python scripts/bench_conv6.py --cfgs 62,70 --batch 1 --hw 135 240 --only conv,convc2,heads,zr" \
 "200 r5y_bench.json python bench.py" \
 "200 r5y_bench_ns4.json env RAFT_FWD6_NS4=1 python bench.py" \
 "200 r5y_bench_b.json python bench.py" \
 "200 r5y_bench_ns4_b.json env RAFT_FWD6_NS4=1 python bench.py" \
 "200 r5y_1080.json $I" \
 "200 r5y_1080_ns4.json env RAFT_FWD6_NS4=1 $I"

#!/bin/bash
# round 5, lease b: 128x64 two-workgroups-per-CU conv_fwd6 tiles (cfg 62/63/64): numerics + timing
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
bash scripts/gpu_step.sh \
 "300 r5b_conv_tests.log $T tests/test_conv_gpu.py -k 'every_variant'" \
 "300 r5b_conv6_c2.log python scripts/bench_conv6.py --cfgs 59,60,61,62,63,64 --only conv,convc2,convf2,fh1,zr,q15,zr51,q51,d_conv,d_fh1,d_zr15,d_q15,d_zr51,d_q51" \
 "300 r5b_conv6_1080.log python scripts/bench_conv6.py --cfgs 59,60,61,62,63,64 --batch 1 --hw 135 240 --only conv,convc2,fh1,zr,q15,zr51,q51" \
 "300 r5b_conv6_sintel.log python scripts/bench_conv6.py --cfgs 59,60,61,62,63,64 --batch 6 --hw 46 96 --only conv,zr,q15,zr51,q51,d_zr51,d_q51"

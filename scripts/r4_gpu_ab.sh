#!/bin/bash
bash scripts/gpu_step.sh \
 "200 r4ab_conv6_1x1.log python scripts/bench_conv6.py --cfgs 41,45 --only convc1,mask2,d_convc1,d_mask2" \
 "200 r4ab_conv6_1x1_1080.log python scripts/bench_conv6.py --cfgs 41,45 --only convc1,mask2,d_convc1,d_mask2 --batch 1 --hw 136 240"

#!/bin/bash
bash scripts/gpu_step.sh \
 "200 r4af_c2.log python scripts/bench_conv6.py --cfgs 41,59,60,61 --only conv,convc2,convf2,fh1,zr51,q51,d_conv,d_fh1,d_zr51,d_q51" \
 "200 r4af_1080.log python scripts/bench_conv6.py --cfgs 41,59,60,61 --only conv,convc2,fh1,zr51,q51 --batch 1 --hw 136 240" \
 "200 r4af_sintel.log python scripts/bench_conv6.py --cfgs 41,59,60,61 --only conv,zr51,q51,d_zr51,d_q51 --batch 6 --hw 46 96"

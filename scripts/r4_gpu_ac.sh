#!/bin/bash
bash scripts/gpu_step.sh \
 "200 r4ac_1x1_blas.log python scripts/bench_1x1_blas.py" \
 "200 r4ac_1x1_blas_1080.log python scripts/bench_1x1_blas.py --batch 1 --hw 136 240"

#!/bin/bash
# round 5, lease t: column-keyed LDS swizzle of the 3x3 2-D halo tiles
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5t_tests.log $T tests/test_conv_gpu.py tests/test_update_fused_gpu.py" \
 "300 r5t_conv6.log python scripts/bench_conv6.py --cfgs 62,63 --only conv,convc2,convf2,heads,d_conv,d_convc2,d_fh1,zr,q15" \
 "300 r5t_conv6_1080.log python scripts/bench_conv6.py --cfgs 62,63 --batch 1 --hw 135 240 --only conv,convc2,heads,zr" \
 "200 r5t_bench.json python bench.py" \
 "200 r5t_bench_b.json python bench.py" \
 "200 r5t_bench_1080.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "300 r5t_pmc.log env PMC_OUT=gpurun_out/r5t_pmc PMC_GROUPS=SQ_INSTS_LDS\ SQ_LDS_BANK_CONFLICT\ SQ_INSTS_MFMA\ GRBM_GUI_ACTIVE\ SQ_VALU_MFMA_BUSY_CYCLES bash scripts/pmc_step.sh"

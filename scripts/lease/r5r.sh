#!/bin/bash
# round 5, lease r: MFMA Cin=8 data gradient (flow-head conv2)
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5r_tests.log $T tests/test_conv_gpu.py -k cin8\ or\ dgrad tests/test_update_fused_gpu.py tests/test_fp16_gpu.py" \
 "200 r5r_bench.json python bench.py" \
 "200 r5r_bench_nocin8.json env RAFT_CIN8=0 python bench.py" \
 "200 r5r_bench_b.json python bench.py" \
 "200 r5r_bench_nocin8_b.json env RAFT_CIN8=0 python bench.py" \
 "300 r5r_pmc.log env PMC_OUT=gpurun_out/r5r_pmc PMC_GROUPS=SQ_WAVES\ SQ_INSTS_MFMA\ GRBM_GUI_ACTIVE bash scripts/pmc_step.sh"

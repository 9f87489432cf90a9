#!/bin/bash
# round 5, lease q: direct Cin=8 data gradient (flow-head conv2); PMC counters of the training step
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5q_tests.log $T tests/test_conv_gpu.py tests/test_update_fused_gpu.py tests/test_fp16_gpu.py" \
 "200 r5q_bench.json python bench.py" \
 "200 r5q_bench_nocin8.json env RAFT_CIN8=0 python bench.py" \
 "200 r5q_bench_b.json python bench.py" \
 "200 r5q_bench_nocin8_b.json env RAFT_CIN8=0 python bench.py" \
 "900 r5q_pmc.log env PMC_OUT=gpurun_out/r5q_pmc bash scripts/pmc_step.sh"

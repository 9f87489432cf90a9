#!/bin/bash
bash scripts/gpu_step.sh \
 "500 r4j_tests.log python -u -m pytest tests/test_update_fused_gpu.py tests/test_split_train_gpu.py tests/test_fp16_gpu.py tests/test_encoder_gpu.py tests/test_golden_gpu.py -x -q --timeout 180 --timeout-method thread" \
 "300 r4j_ddp.log python -u -m pytest tests/test_ddp_gpu.py -q -s --timeout 300 --timeout-method thread" \
 "200 r4j_lead.log python scripts/host_lead.py --steps 20" \
 "150 r4j_bench_a.json python bench.py --steps 30" \
 "150 r4j_bench_hp.json env RAFT_HP_MAIN=1 python bench.py --steps 30" \
 "150 r4j_bench_a2.json python bench.py --steps 30" \
 "150 r4j_bench_hp2.json env RAFT_HP_MAIN=1 python bench.py --steps 30" \
 "200 r4j_bench_fp32.json python bench.py --fp32 --steps 10" \
 "200 r4j_bench_fp16.json python bench.py --amp_dtype fp16 --steps 20"

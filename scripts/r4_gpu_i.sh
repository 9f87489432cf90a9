#!/bin/bash
bash scripts/gpu_step.sh \
 "200 r4i_lead.log python scripts/host_lead.py --steps 20 --max_lead 1" \
 "400 r4i_pack_test.log python -u -m pytest tests/test_pack_multi_gpu.py tests/test_split_train_gpu.py tests/test_update_fused_gpu.py -x -q --timeout 180 --timeout-method thread" \
 "150 r4i_bench.json python bench.py --steps 30" \
 "200 r4i_bench_fp32.json python bench.py --fp32 --steps 10"

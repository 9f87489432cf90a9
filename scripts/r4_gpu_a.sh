#!/bin/bash
# round-4 GPU session A: fp32 split diagnostics + tests, fp16 tests, profiles, bench A/Bs
bash scripts/gpu_step.sh \
 "300 r4_diag.log python -u scripts/diag_split_grads.py" \
 "400 r4_split_test2.log python -u -m pytest tests/test_split_train_gpu.py tests/test_fp16_gpu.py -v -s --timeout 120 --timeout-method thread" \
 "200 r4_bench_q4.json python bench.py" \
 "200 r4_bench_noearly.json env RAFT_EARLY_WGRAD=0 python bench.py" \
 "200 r4_bench_q8.json env GPU_MAX_HW_QUEUES=8 python bench.py" \
 "200 r4_bench_hp.json env RAFT_HP_MAIN=1 python bench.py" \
 "200 r4_bench_fp16.json python bench.py --amp_dtype fp16" \
 "200 r4_bench_corrfp32.json python bench.py --corr_fp32" \
 "200 r4_bench_fp32.json python bench.py --fp32 --steps 10 --warmup 3" \
 "300 r4_prof_fp32.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp32 -o run -- python3 bench.py --fp32 --steps 4 --warmup 2" \
 "300 r4_ddp_nccl.log python -u -m pytest tests/test_ddp_gpu.py -v -s -k nccl --timeout 300 --timeout-method thread"

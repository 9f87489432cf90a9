#!/bin/bash
# round-4 GPU session C: fixed fp32 / DDP tests, host-issue vs GPU time, graph / stream A/Bs, idle-gap listing
S="python scripts/rocpd_summary.py"
C="python scripts/rocpd_concurrency.py"
bash scripts/gpu_step.sh \
 "500 r4c_tests.log python -u -m pytest tests/test_split_train_gpu.py tests/test_golden_gpu.py -v -s --timeout 180 --timeout-method thread -k 'small or lookup or fp32_training'" \
 "300 r4c_ddp.log python -u -m pytest tests/test_ddp_gpu.py -v -s -k nccl --timeout 300 --timeout-method thread" \
 "200 r4c_cpu_issue.log python scripts/cpu_issue.py --steps 5" \
 "150 r4c_bench_a.json python bench.py --steps 30" \
 "150 r4c_bench_graph.json python bench.py --steps 30 --graph" \
 "150 r4c_bench_split2.json env RAFT_WGRAD_SPLIT=2 python bench.py --steps 30" \
 "150 r4c_bench_hp_split2.json env RAFT_HP_MAIN=1 RAFT_WGRAD_SPLIT=2 python bench.py --steps 30" \
 "150 r4c_bench_hp.json env RAFT_HP_MAIN=1 python bench.py --steps 30" \
 "150 r4c_bench_a2.json python bench.py --steps 30" \
 "300 r4c_prof_bf16.log rocprofv3 --kernel-trace -d gpurun_out/pc -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r4c_bf16_concurrency.txt $C gpurun_out/pc/run_results.db --boundary seq_loss_fwd --steps 3 --top 30 --gaps 60" \
 "30 r4c_rm.log rm -rf gpurun_out/pc"

#!/bin/bash
S="python scripts/rocpd_summary.py"
C="python scripts/rocpd_concurrency.py"
bash scripts/gpu_step.sh \
 "150 r4m_bench_a.json python bench.py --steps 30" \
 "150 r4m_bench_mt2.json env RAFT_WGRAD3_MT=2 python bench.py --steps 30" \
 "150 r4m_bench_ws2.json env RAFT_WGRAD_STREAMS=2 python bench.py --steps 30" \
 "150 r4m_bench_nolead.json env RAFT_MAX_LEAD=0 python bench.py --steps 30" \
 "150 r4m_bench_a2.json python bench.py --steps 30" \
 "150 r4m_bench_mt2b.json env RAFT_WGRAD3_MT=2 python bench.py --steps 30" \
 "150 r4m_bench_ws2b.json env RAFT_WGRAD_STREAMS=2 python bench.py --steps 30" \
 "150 r4m_bench_nolead2.json env RAFT_MAX_LEAD=0 python bench.py --steps 30" \
 "200 r4m_convs_mt1.log python scripts/bench_convs.py" \
 "200 r4m_convs_mt2.log env RAFT_WGRAD3_MT=2 python scripts/bench_convs.py" \
 "300 r4m_prof_bf16.log rocprofv3 --kernel-trace -d gpurun_out/pm -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r4m_bf16_kernels.txt $S gpurun_out/pm/run_results.db --boundary seq_loss_fwd --steps 3 --top 60" \
 "120 r4m_bf16_concurrency.txt $C gpurun_out/pm/run_results.db --boundary seq_loss_fwd --steps 3 --top 30 --gaps 40" \
 "30 r4m_rm.log rm -rf gpurun_out/pm" \
 "200 r4m_bench_1080.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3"

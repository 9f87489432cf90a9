#!/bin/bash
# round 5, lease j: lean 1x1 GEMM (v7) numerics + A/B; alt-corr fill fix; graph-replay concurrency; host issue
S="python scripts/rocpd_summary.py"
C="python scripts/rocpd_concurrency.py"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "400 r5j_tests.log $T tests/test_conv_gpu.py tests/test_update_fused_gpu.py tests/test_kernels_gpu.py" \
 "300 r5j_conv1x1.log python scripts/bench_conv6.py --cfgs 8,67 --only convc1,mask2,d_convc1,d_mask2" \
 "300 r5j_conv1x1_1080.log python scripts/bench_conv6.py --cfgs 8,67 --batch 1 --hw 135 240 --only convc1,mask2,d_convc1,d_mask2" \
 "200 r5j_bench_v7.json python bench.py" \
 "200 r5j_bench_v4.json env RAFT_CONV_V7=0 python bench.py" \
 "200 r5j_bench_v7b.json python bench.py" \
 "200 r5j_bench_v4b.json env RAFT_CONV_V7=0 python bench.py" \
 "200 r5j_bench_1080.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "200 r5j_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "200 r5j_host_lead.log python scripts/host_lead.py --steps 20 --hp" \
 "300 r5j_prof_graph.log rocprofv3 --kernel-trace -d gpurun_out/pg -o run -- python3 bench.py --graph --steps 4 --warmup 3" \
 "120 r5j_graph_kernels.txt $S gpurun_out/pg/run_results.db --boundary seq_loss_fwd --steps 3 --top 20" \
 "120 r5j_graph_concurrency.txt $C gpurun_out/pg/run_results.db --boundary seq_loss_fwd --steps 3 --top 20 --gaps 30" \
 "30 r5j_rm.log rm -rf gpurun_out/pg"

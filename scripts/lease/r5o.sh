#!/bin/bash
# round 5, lease o: native step executor (fused_step_fwd); 8-wave 5-tap weight gradients; corr v3 default
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "500 r5o_tests.log $T tests/test_update_fused_gpu.py tests/test_model_gpu.py tests/test_fp16_gpu.py tests/test_golden_gpu.py tests/test_train_graph.py tests/test_kernels_gpu.py tests/test_conv_gpu.py" \
 "200 r5o_host_lead.log python scripts/host_lead.py --steps 20 --hp" \
 "200 r5o_host_lead_py.log env RAFT_NATIVE_STEP=0 python scripts/host_lead.py --steps 20 --hp" \
 "200 r5o_bench_native.json python bench.py" \
 "200 r5o_bench_py.json env RAFT_NATIVE_STEP=0 python bench.py" \
 "200 r5o_bench_mt2.json env RAFT_WGRAD3_MT=2 python bench.py" \
 "200 r5o_bench_native_b.json python bench.py" \
 "200 r5o_bench_py_b.json env RAFT_NATIVE_STEP=0 python bench.py" \
 "200 r5o_bench_mt2_b.json env RAFT_WGRAD3_MT=2 python bench.py" \
 "200 r5o_bench_1080.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "200 r5o_bench_1080_py.json env RAFT_NATIVE_STEP=0 python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "200 r5o_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "300 r5o_prof_bf16.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r5o_bf16_kernels.txt python scripts/rocpd_summary.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 60" \
 "30 r5o_rm.log rm -rf gpurun_out/pk"

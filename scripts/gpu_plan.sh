#!/bin/bash
# The current GPU session plan (one gpurun call): steps run in order by scripts/gpu_step.sh,
# each "<timeout s> <log under gpurun_out/> <command>"; the first crash / time-out ends it.
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
bash scripts/gpu_step.sh \
 "600 r6c_tests.log $T tests/test_kernels_gpu.py tests/test_conv_gpu.py tests/test_update_fused_gpu.py tests/test_golden_gpu.py tests/test_encoder_gpu.py" \
 "200 r6c_bench.json python bench.py" \
 "200 r6c_bench_blas.json env RAFT_CORR_BWD_BLAS=1 python bench.py" \
 "200 r6c_bench2.json python bench.py" \
 "200 r6c_bench_graph.json python bench.py --graph" \
 "200 r6c_b1_368x768.json python bench.py --batch 1 --image_size 368 768" \
 "200 r6c_b1_368x768_graph.json python bench.py --batch 1 --image_size 368 768 --graph" \
 "200 r6c_b2_368x768_graph.json python bench.py --batch 2 --image_size 368 768 --graph" \
 "200 r6c_b1_400x720_graph.json python bench.py --batch 1 --image_size 400 720 --graph" \
 "200 r6c_b2_400x720_graph.json python bench.py --batch 2 --image_size 400 720 --graph" \
 "300 r6c_prof.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r6c_kernels.txt python scripts/rocpd_summary.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 60" \
 "30 r6c_rm.log rm -rf gpurun_out/pk"

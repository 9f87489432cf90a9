#!/bin/bash
# round 5, lease x: batched weight gradients issued at the end of the loop backward
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "400 r5x_tests.log $T tests/test_update_fused_gpu.py tests/test_model_gpu.py tests/test_golden_gpu.py tests/test_ddp_gpu.py tests/test_train_graph.py tests/test_fp16_gpu.py" \
 "200 r5x_bench.json python bench.py" \
 "200 r5x_bench_old.json env RAFT_WGRAD_AT_LOOP_END=0 python bench.py" \
 "200 r5x_bench_b.json python bench.py" \
 "200 r5x_bench_old_b.json env RAFT_WGRAD_AT_LOOP_END=0 python bench.py" \
 "200 r5x_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "200 r5x_bench_alt_old.json env RAFT_WGRAD_AT_LOOP_END=0 python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "300 r5x_prof.log rocprofv3 --kernel-trace -d gpurun_out/pw -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r5x_phases.txt python scripts/step_phases.py gpurun_out/pw/run_results.db --top 6" \
 "30 r5x_rm.log rm -rf gpurun_out/pw"

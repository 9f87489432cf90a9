#!/bin/bash
# round 5, lease l: flow_head.conv2 folded into the heads conv epilogue (numerics + A/B)
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5l_tests.log $T tests/test_conv_gpu.py -k flow_head_conv2 tests/test_update_fused_gpu.py tests/test_model_gpu.py" \
 "200 r5l_bench_fold.json python bench.py" \
 "200 r5l_bench_nofold.json env RAFT_FOLD_N2=0 python bench.py" \
 "200 r5l_bench_fold_b.json python bench.py" \
 "200 r5l_bench_nofold_b.json env RAFT_FOLD_N2=0 python bench.py" \
 "200 r5l_bench_1080_fold.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "200 r5l_bench_1080_nofold.json env RAFT_FOLD_N2=0 python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "300 r5l_prof_1080.log rocprofv3 --kernel-trace -d gpurun_out/p1080 -o run -- python3 bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 4 --warmup 2" \
 "120 r5l_1080_kernels.txt python scripts/rocpd_summary.py gpurun_out/p1080/run_results.db --boundary corr_volume --steps 3 --top 30" \
 "30 r5l_rm.log rm -rf gpurun_out/p1080"

#!/bin/bash
# round 5, lease z: encoder prepack inside the inference graph
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
I="python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "400 r5z_tests.log $T tests/test_model_gpu.py tests/test_encoder_gpu.py tests/test_golden_gpu.py" \
 "200 r5z_1080.json $I" \
 "200 r5z_1080_noprepack.json env RAFT_ENC_PREPACK=0 $I" \
 "200 r5z_1080_b.json $I" \
 "200 r5z_1080_noprepack_b.json env RAFT_ENC_PREPACK=0 $I" \
 "200 r5z_ros_fp32.json python bench.py --mode infer --fp32 --image_size 440 1024 --iters 20 --batch 1 --steps 20 --warmup 3" \
 "200 r5z_sintel.json python bench.py --mode infer --image_size 440 1024 --iters 32 --batch 1 --steps 20 --warmup 3" \
 "300 r5z_prof_1080.log rocprofv3 --kernel-trace -d gpurun_out/p1080 -o run -- python3 bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 4 --warmup 2" \
 "120 r5z_1080_kernels.txt python scripts/rocpd_summary.py gpurun_out/p1080/run_results.db --boundary corr_volume --steps 3 --top 30" \
 "30 r5z_rm.log rm -rf gpurun_out/p1080"

#!/bin/bash
# round 5, lease al: one-branch norm-backward apply at six waves per SIMD
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "400 r5al_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_encoder_gpu.py tests/test_golden_gpu.py tests/test_fp16_gpu.py tests/test_split_train_gpu.py tests/test_ddp_gpu.py" \
 "200 r5al_bench.json python bench.py" \
 "200 r5al_bench_b.json python bench.py" \
 "300 r5al_prof.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r5al_kernels.txt python scripts/rocpd_summary.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 80" \
 "30 r5al_rm.log rm -rf gpurun_out/pk"

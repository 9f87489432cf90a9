#!/bin/bash
# round 5, lease ak: convex-upsampling backward with fewer live registers
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "400 r5ak_tests.log python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_update_fused_gpu.py tests/test_golden_gpu.py tests/test_fp16_gpu.py" \
 "200 r5ak_bench.json python bench.py" \
 "200 r5ak_bench_b.json python bench.py" \
 "300 r5ak_prof.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r5ak_kernels.txt python scripts/rocpd_summary.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 80" \
 "30 r5ak_rm.log rm -rf gpurun_out/pk"

#!/bin/bash
S="python scripts/rocpd_summary.py"
bash scripts/gpu_step.sh \
 "500 r4u_tests.log python -u -m pytest tests/test_split_train_gpu.py tests/test_golden_gpu.py tests/test_conv_gpu.py tests/test_update_fused_gpu.py tests/test_fp16_gpu.py -q -s --timeout 300 --timeout-method thread" \
 "200 r4u_bench_fp32.json python bench.py --fp32 --steps 10" \
 "200 r4u_bench_fp32b.json python bench.py --fp32 --steps 10" \
 "200 r4u_bench_small_fp32.json python bench.py --fp32 --small --steps 10" \
 "300 r4u_prof_fp32.log rocprofv3 --kernel-trace -d gpurun_out/pf -o run -- python3 bench.py --fp32 --steps 4 --warmup 2" \
 "120 r4u_fp32_kernels.txt $S gpurun_out/pf/run_results.db --boundary seq_loss_fwd --steps 3 --top 90" \
 "30 r4u_rm.log rm -rf gpurun_out/pf"

#!/bin/bash
# round 5, lease m: planar folded flow-head partials; direct 7x7 convf1 kernel
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5m_tests.log $T tests/test_conv_gpu.py tests/test_update_fused_gpu.py tests/test_model_gpu.py tests/test_fp16_gpu.py" \
 "200 r5m_bench.json python bench.py" \
 "200 r5m_bench_b.json python bench.py" \
 "200 r5m_bench_1080.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "300 r5m_prof_1080.log rocprofv3 --kernel-trace -d gpurun_out/p1080 -o run -- python3 bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 4 --warmup 2" \
 "120 r5m_1080_kernels.txt python scripts/rocpd_summary.py gpurun_out/p1080/run_results.db --boundary corr_volume --steps 3 --top 30" \
 "30 r5m_rm.log rm -rf gpurun_out/p1080" \
 "300 r5m_prof_bf16.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r5m_bf16_kernels.txt python scripts/rocpd_summary.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 60" \
 "120 r5m_bf16_concurrency.txt python scripts/rocpd_concurrency.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 30 --gaps 40" \
 "30 r5m_rm2.log rm -rf gpurun_out/pk" \
 "200 r5m_host_cprofile.log python scripts/host_lead.py --steps 20 --hp --cprofile 10"

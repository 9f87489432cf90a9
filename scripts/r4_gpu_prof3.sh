#!/bin/bash
S="python scripts/rocpd_summary.py"
C="python scripts/rocpd_concurrency.py"
bash scripts/gpu_step.sh \
 "300 r4p3_prof_bf16.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r4p3_bf16_kernels.txt $S gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 60" \
 "120 r4p3_bf16_concurrency.txt $C gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 30 --gaps 40" \
 "30 r4p3_rm.log rm -rf gpurun_out/pk" \
 "300 r4p3_prof_1080.log rocprofv3 --kernel-trace -d gpurun_out/p1 -o run -- python3 bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 3 --warmup 2" \
 "120 r4p3_1080_kernels.txt $S gpurun_out/p1/run_results.db --boundary corr_volume --steps 3 --top 40" \
 "30 r4p3_rm2.log rm -rf gpurun_out/p1"

#!/bin/bash
# round 5, lease s: kernel profiles of the fp32 training step and the alternate-corr step; graph replay profile
S="python scripts/rocpd_summary.py"
C="python scripts/rocpd_concurrency.py"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "200 r5s_bench_fp32.json python bench.py --fp32 --steps 10" \
 "300 r5s_prof_fp32.log rocprofv3 --kernel-trace -d gpurun_out/pf -o run -- python3 bench.py --fp32 --steps 4 --warmup 2" \
 "120 r5s_fp32_kernels.txt $S gpurun_out/pf/run_results.db --boundary seq_loss_fwd --steps 3 --top 40" \
 "120 r5s_fp32_concurrency.txt $C gpurun_out/pf/run_results.db --boundary seq_loss_fwd --steps 3 --top 20 --gaps 20" \
 "30 r5s_rm1.log rm -rf gpurun_out/pf" \
 "300 r5s_prof_alt.log rocprofv3 --kernel-trace -d gpurun_out/pa -o run -- python3 bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 4 --warmup 2" \
 "120 r5s_alt_kernels.txt $S gpurun_out/pa/run_results.db --boundary seq_loss_fwd --steps 3 --top 40" \
 "120 r5s_alt_concurrency.txt $C gpurun_out/pa/run_results.db --boundary seq_loss_fwd --steps 3 --top 20 --gaps 20" \
 "30 r5s_rm2.log rm -rf gpurun_out/pa"

#!/bin/bash
S="python scripts/rocpd_summary.py"
bash scripts/gpu_step.sh \
 "300 r4t_prof_fp32.log rocprofv3 --kernel-trace -d gpurun_out/pf -o run -- python3 bench.py --fp32 --steps 4 --warmup 2" \
 "120 r4t_fp32_kernels.txt $S gpurun_out/pf/run_results.db --boundary seq_loss_fwd --steps 3 --top 90" \
 "30 r4t_rm.log rm -rf gpurun_out/pf"

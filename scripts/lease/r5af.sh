#!/bin/bash
# round 5, lease af: kernel table with the pyramid backward GEMMs on hipBLASLt
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5af_prof.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r5af_kernels.txt python scripts/rocpd_summary.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 80" \
 "30 r5af_rm.log rm -rf gpurun_out/pk"

#!/bin/bash
# round 5, lease am: 1080p inference kernel table on the end-of-round tree
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5am_prof_1080.log rocprofv3 --kernel-trace -d gpurun_out/p1080 -o run -- python3 bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 4 --warmup 2" \
 "120 r5am_1080_kernels.txt python scripts/rocpd_summary.py gpurun_out/p1080/run_results.db --boundary corr_volume --steps 3 --top 30" \
 "30 r5am_rm.log rm -rf gpurun_out/p1080"

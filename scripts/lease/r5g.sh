#!/bin/bash
# round 5, lease g: gather backward v2 (wave-aggregated binning, LDS tap gradients) + by-grid step profile
S="python scripts/rocpd_summary.py"
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5g_tests.log $T tests/test_kernels_gpu.py -k 'local_corr or deterministic'" \
 "200 r5g_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "200 r5g_bench_alt_old.json env RAFT_LC_GATHER=0 python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "300 r5g_prof_alt.log rocprofv3 --kernel-trace -d gpurun_out/pa -o run -- python3 bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 4 --warmup 3" \
 "120 r5g_alt_kernels.txt $S gpurun_out/pa/run_results.db --boundary seq_loss_fwd --steps 3 --top 40" \
 "30 r5g_rm.log rm -rf gpurun_out/pa" \
 "300 r5g_prof_bf16.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r5g_bf16_by_grid.txt $S gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 70 --by-grid" \
 "30 r5g_rm2.log rm -rf gpurun_out/pk"

#!/bin/bash
# round 5, lease h: sharded binning for the gather backward; wide-N 1x1 GEMM tiles
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
S="python scripts/rocpd_summary.py"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5h_tests.log $T tests/test_kernels_gpu.py -k 'local_corr or deterministic'" \
 "200 r5h_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "300 r5h_conv1x1.log python scripts/bench_conv6.py --cfgs 8,70,71 --only convc1,mask2,d_convc1,d_mask2" \
 "300 r5h_conv1x1_1080.log python scripts/bench_conv6.py --cfgs 8,70,71 --batch 1 --hw 135 240 --only convc1,mask2,d_convc1,d_mask2" \
 "300 r5h_prof_alt.log rocprofv3 --kernel-trace -d gpurun_out/pa -o run -- python3 bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 4 --warmup 3" \
 "120 r5h_alt_kernels.txt $S gpurun_out/pa/run_results.db --boundary seq_loss_fwd --steps 3 --top 30" \
 "30 r5h_rm.log rm -rf gpurun_out/pa"
bash scripts/gpu_step.sh \
 "300 r5h_fh2.log python scripts/bench_conv6.py --cfgs 41,59,62 --only fh2" \
 "300 r5h_fh2_1080.log python scripts/bench_conv6.py --cfgs 59,62 --batch 1 --hw 135 240 --only fh2" \
 "200 r5h_bench_graph.json python bench.py --graph" \
 "200 r5h_bench_eager.json python bench.py --no-graph"

#!/bin/bash
# round 5, final (second pass, after the hipBLASLt pyramid backward and the encoder occupancy work): full GPU suite, smoke, the configs' benches on the end-of-round tree
T="python -u -m pytest tests -m gpu -q -rf --tb=short --timeout 200 --timeout-method thread"
I="python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "900 r5g2_gputests.log $T" \
 "300 r5g2_smoke.log python -c 'import __graft_entry__ as g; g.smoke()'" \
 "200 r5g2_bench_a.json python bench.py" \
 "200 r5g2_bench_1080_a.json $I" \
 "200 r5g2_bench_b.json python bench.py" \
 "200 r5g2_bench_1080_b.json $I" \
 "200 r5g2_bench_c.json python bench.py --steps 40" \
 "300 r5g2_prof.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r5g2_kernels.txt python scripts/rocpd_summary.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 80" \
 "30 r5g2_rm.log rm -rf gpurun_out/pk" \
 "200 r5g2_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "200 r5g2_bench_kitti_dense.json python bench.py --batch 3 --image_size 376 1248 --steps 15" \
 "200 r5g2_bench_sintel.json python bench.py --batch 6 --image_size 368 768" \
 "200 r5g2_bench_full.json python bench.py --batch 6 --image_size 440 1024 --steps 15" \
 "200 r5g2_bench_fp16.json python bench.py --amp_dtype fp16" \
 "200 r5g2_bench_fp32.json python bench.py --fp32 --steps 10" \
 "200 r5g2_bench_infer_sintel.json python bench.py --mode infer --image_size 440 1024 --iters 32 --batch 1 --steps 20 --warmup 3" \
 "200 r5g2_bench_ros_fp32.json python bench.py --mode infer --fp32 --image_size 440 1024 --iters 20 --batch 1 --steps 20 --warmup 3" \
 "200 r5g2_bench_small.json python bench.py --small"

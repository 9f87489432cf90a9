#!/bin/bash
# The current GPU session plan (one gpurun call): steps run in order by scripts/gpu_step.sh,
# each "<timeout s> <log under gpurun_out/> <command>"; the first crash / time-out ends it.
# (This one: the round's configuration sweep -- full GPU suite, smoke, every config's bench.)
export TMPDIR=/tmp
T="python -u -m pytest tests -m gpu -q -rf --tb=short --timeout 200 --timeout-method thread"
I="python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3"
P=r6s
bash scripts/gpu_step.sh \
 "900 ${P}_gputests.log $T" \
 "300 ${P}_smoke.log python -c 'import __graft_entry__ as g; g.smoke()'" \
 "200 ${P}_bench_a.json python bench.py" \
 "200 ${P}_bench_1080_a.json $I" \
 "200 ${P}_bench_b.json python bench.py" \
 "200 ${P}_bench_1080_b.json $I" \
 "200 ${P}_bench_c.json python bench.py --steps 40" \
 "200 ${P}_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "200 ${P}_bench_kitti_dense.json python bench.py --batch 3 --image_size 376 1248 --steps 15" \
 "200 ${P}_bench_sintel.json python bench.py --batch 6 --image_size 368 768" \
 "200 ${P}_bench_full.json python bench.py --batch 6 --image_size 440 1024 --steps 15" \
 "200 ${P}_bench_fp16.json python bench.py --amp_dtype fp16" \
 "200 ${P}_bench_fp32.json python bench.py --fp32 --steps 10" \
 "200 ${P}_bench_infer_sintel.json python bench.py --mode infer --image_size 440 1024 --iters 32 --batch 1 --steps 20 --warmup 3" \
 "200 ${P}_bench_ros_fp32.json python bench.py --mode infer --fp32 --image_size 440 1024 --iters 20 --batch 1 --steps 20 --warmup 3" \
 "200 ${P}_bench_small.json python bench.py --small" \
 "200 ${P}_b1_368x768.json python bench.py --batch 1 --image_size 368 768 --steps 40" \
 "200 ${P}_b1_368x768_graph.json python bench.py --batch 1 --image_size 368 768 --steps 40 --graph" \
 "200 ${P}_b2_368x768.json python bench.py --batch 2 --image_size 368 768 --steps 40" \
 "200 ${P}_b2_368x768_graph.json python bench.py --batch 2 --image_size 368 768 --steps 40 --graph" \
 "200 ${P}_b1_400x720.json python bench.py --batch 1 --image_size 400 720 --steps 40" \
 "200 ${P}_b1_400x720_graph.json python bench.py --batch 1 --image_size 400 720 --steps 40 --graph" \
 "200 ${P}_b2_400x720.json python bench.py --batch 2 --image_size 400 720 --steps 40" \
 "200 ${P}_b2_400x720_graph.json python bench.py --batch 2 --image_size 400 720 --steps 40 --graph" \
 "200 ${P}_b6_400x720.json python bench.py --batch 6 --image_size 400 720"

#!/bin/bash
# round 5, lease n: corr volume v3 (BK 32, 4 WG/CU, swapped-operand epilogue); n2_apply branch-free;
# graphed train step without the flat gradient buffer, on the high-priority stream
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5n_tests.log $T tests/test_kernels_gpu.py tests/test_conv_gpu.py -k corr_volume_v2_matches_generic\ or\ flow_head_conv2" \
 "300 r5n_bench_corr.log python scripts/bench_corr.py" \
 "200 r5n_bench_1080.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "300 r5n_graph_tests.log $T tests/test_train_graph.py" \
 "200 r5n_bench_graph.json python bench.py --graph" \
 "200 r5n_bench_eager.json python bench.py" \
 "200 r5n_bench_graph_flat.json env RAFT_GRAPH_FLAT=1 python bench.py --graph" \
 "200 r5n_bench_graph_nohp.json env RAFT_GRAPH_HP=0 python bench.py --graph" \
 "200 r5n_bench_graph2.json python bench.py --graph" \
 "200 r5n_bench_eager2.json python bench.py"

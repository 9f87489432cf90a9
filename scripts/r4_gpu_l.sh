#!/bin/bash
bash scripts/gpu_step.sh \
 "400 r4l_enc_lookup_tests.log python -u -m pytest tests/test_encoder_gpu.py tests/test_kernels_gpu.py tests/test_golden_gpu.py -x -q --timeout 180 --timeout-method thread" \
 "300 r4l_wgrad_mt2_tests.log env RAFT_WGRAD3_MT=2 python -u -m pytest tests/test_conv_gpu.py tests/test_update_fused_gpu.py -x -q -k wgrad --timeout 180 --timeout-method thread" \
 "300 r4l_streams2_tests.log env RAFT_WGRAD_STREAMS=2 python -u -m pytest tests/test_update_fused_gpu.py -x -q --timeout 180 --timeout-method thread" \
 "200 r4l_convs_mt1.log python scripts/bench_convs.py" \
 "200 r4l_convs_mt2.log env RAFT_WGRAD3_MT=2 python scripts/bench_convs.py" \
 "150 r4l_bench_a.json python bench.py --steps 30" \
 "150 r4l_bench_mt2.json env RAFT_WGRAD3_MT=2 python bench.py --steps 30" \
 "150 r4l_bench_ws2.json env RAFT_WGRAD_STREAMS=2 python bench.py --steps 30" \
 "150 r4l_bench_a2.json python bench.py --steps 30" \
 "150 r4l_bench_mt2b.json env RAFT_WGRAD3_MT=2 python bench.py --steps 30" \
 "150 r4l_bench_ws2b.json env RAFT_WGRAD_STREAMS=2 python bench.py --steps 30"

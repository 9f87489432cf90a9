#!/bin/bash
# round 5, lease ae: pyramid backward GEMMs on hipBLASLt vs the generic MFMA GEMM
bash scripts/gpu_step.sh \
 "300 r5ae_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_golden_gpu.py tests/test_model_gpu.py tests/test_update_fused_gpu.py tests/test_query_shard_gpu.py" \
 "200 r5ae_blas.json python bench.py" \
 "200 r5ae_mfma.json env RAFT_CORR_BWD_BLAS=0 python bench.py" \
 "200 r5ae_blasb.json python bench.py" \
 "200 r5ae_mfmab.json env RAFT_CORR_BWD_BLAS=0 python bench.py"

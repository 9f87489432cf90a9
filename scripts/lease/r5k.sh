#!/bin/bash
# round 5, lease k: conv forward variants incl. the lean 1x1 GEMM (v7) after the oracle fix
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "500 r5k_tests.log $T tests/test_conv_gpu.py tests/test_update_fused_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py"

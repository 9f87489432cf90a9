#!/bin/bash
# round 5, lease ah: deferred lookup backward with batched neighbour RMW
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5ah_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_golden_gpu.py tests/test_model_gpu.py tests/test_update_fused_gpu.py" \
 "200 r5ah_br.json python bench.py" \
 "200 r5ah_rmw.json env RAFT_GRAD_ROWS_BATCH=0 python bench.py" \
 "200 r5ah_brb.json python bench.py" \
 "200 r5ah_rmwb.json env RAFT_GRAD_ROWS_BATCH=0 python bench.py" \
 "300 r5ah_prof.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r5ah_kernels.txt python scripts/rocpd_summary.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 80" \
 "30 r5ah_rm.log rm -rf gpurun_out/pk"

#!/bin/bash
# round 5, lease ab: local correlation with prefetched slice staging and transposed dF1 fragments
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
A="python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "400 r5ab_tests.log $T tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_update_fused_gpu.py" \
 "200 r5ab_alt.json $A" \
 "200 r5ab_alt_b.json $A" \
 "300 r5ab_prof_alt.log rocprofv3 --kernel-trace -d gpurun_out/pa -o run -- python3 bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 4 --warmup 2" \
 "120 r5ab_alt_kernels.txt python scripts/rocpd_summary.py gpurun_out/pa/run_results.db --boundary seq_loss_fwd --steps 3 --top 25" \
 "30 r5ab_rm.log rm -rf gpurun_out/pa"

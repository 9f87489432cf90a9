#!/bin/bash
# round 5, lease f: gather-form --alternate_corr backward (numerics + A/B) and the GradSync DDP GPU tests
S="python scripts/rocpd_summary.py"
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "400 r5f_tests.log $T tests/test_kernels_gpu.py -k 'local_corr or deterministic' tests/test_ddp_gpu.py tests/test_model_gpu.py -k 'alternate or local_corr or deterministic or ddp or rccl'" \
 "200 r5f_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "200 r5f_bench_alt_old.json env RAFT_LC_GATHER=0 python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "200 r5f_bench_alt2.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "300 r5f_prof_alt.log rocprofv3 --kernel-trace -d gpurun_out/pa -o run -- python3 bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 4 --warmup 3" \
 "120 r5f_alt_kernels.txt $S gpurun_out/pa/run_results.db --boundary seq_loss_fwd --steps 3 --top 40" \
 "30 r5f_rm.log rm -rf gpurun_out/pa"

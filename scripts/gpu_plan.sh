#!/bin/bash
# The current GPU session plan (one gpurun call): steps run in order by scripts/gpu_step.sh,
# each "<timeout s> <log under gpurun_out/> <command>"; the first crash / time-out ends it.
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
bash scripts/gpu_step.sh \
 "300 r6l_tests.log env RAFT_WGRAD2_STAGES=2 $T tests/test_conv_gpu.py -k wgrad" \
 "200 r6l_base.json python bench.py" \
 "200 r6l_s2.json env RAFT_WGRAD2_STAGES=2 python bench.py" \
 "200 r6l_mt1.json env RAFT_WGRAD3_MT=1 python bench.py" \
 "200 r6l_base_b.json python bench.py" \
 "200 r6l_s2_b.json env RAFT_WGRAD2_STAGES=2 python bench.py" \
 "200 r6l_mt1_b.json env RAFT_WGRAD3_MT=1 python bench.py" \
 "300 r6l_prof.log env RAFT_WGRAD2_STAGES=2 rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r6l_kernels.txt python scripts/rocpd_summary.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 40" \
 "30 r6l_rm.log rm -rf gpurun_out/pk"

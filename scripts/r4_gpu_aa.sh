#!/bin/bash
S="python scripts/rocpd_summary.py"
C="python scripts/rocpd_concurrency.py"
bash scripts/gpu_step.sh \
 "300 r4aa_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_encoder_gpu.py tests/test_model_gpu.py tests/test_golden_gpu.py" \
 "150 r4aa_a1.json python bench.py --steps 40" \
 "150 r4aa_np1.json env RAFT_ENC_PREPACK=0 python bench.py --steps 40" \
 "150 r4aa_fk1.json env RAFT_ENC_PREPACK=fork python bench.py --steps 40" \
 "150 r4aa_a2.json python bench.py --steps 40" \
 "150 r4aa_np2.json env RAFT_ENC_PREPACK=0 python bench.py --steps 40" \
 "150 r4aa_fk2.json env RAFT_ENC_PREPACK=fork python bench.py --steps 40" \
 "200 r4aa_f1.json python bench.py --steps 20 --fp32" \
 "200 r4aa_fn1.json env RAFT_ENC_PREPACK=0 python bench.py --steps 20 --fp32" \
 "300 r4aa_prof_bf16.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r4aa_bf16_kernels.txt $S gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 60" \
 "120 r4aa_bf16_concurrency.txt $C gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 30 --gaps 40" \
 "30 r4aa_rm.log rm -rf gpurun_out/pk"

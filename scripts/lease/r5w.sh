#!/bin/bash
# round 5, lease w: phases of the training step (forward / loop backward / tail / optimizer)
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5w_prof.log rocprofv3 --kernel-trace -d gpurun_out/pw -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r5w_phases.txt python scripts/step_phases.py gpurun_out/pw/run_results.db --top 6" \
 "120 r5w_concurrency.txt python scripts/rocpd_concurrency.py gpurun_out/pw/run_results.db --boundary seq_loss_fwd --steps 3 --top 20 --gaps 20" \
 "30 r5w_rm.log rm -rf gpurun_out/pw"

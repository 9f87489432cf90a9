#!/bin/bash
# round 5, lease ac: where the batched weight gradients sit in the unprofiled step
bash scripts/gpu_step.sh \
 "200 r5ac_wgrad_timing.log python scripts/host_lead.py --steps 20 --hp --wgrad_timing" \
 "200 r5ac_wgrad_timing_mt3.log env RAFT_WGRAD3_MT=3 python scripts/host_lead.py --steps 20 --hp --wgrad_timing" \
 "200 r5ac_wgrad_timing_early.log env RAFT_WGRAD_AT_LOOP_END=1 python scripts/host_lead.py --steps 20 --hp"

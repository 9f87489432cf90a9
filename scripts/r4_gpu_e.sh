#!/bin/bash
bash scripts/gpu_step.sh \
 "120 r4e_queue_depth.log python scripts/queue_depth.py --n 3000" \
 "120 r4e_queue_depth_q8.log env GPU_MAX_HW_QUEUES=8 python scripts/queue_depth.py --n 3000"

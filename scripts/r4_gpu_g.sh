#!/bin/bash
bash scripts/gpu_step.sh \
 "200 r4g_lead_gpupad.log python scripts/host_lead.py --steps 20 --gpu_pad_ms 3" \
 "200 r4g_lead_hostpad.log python scripts/host_lead.py --steps 20 --host_pad_ms 2"

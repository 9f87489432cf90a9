#!/bin/bash
bash scripts/gpu_step.sh \
 "200 r4h_lead40.log python scripts/host_lead.py --steps 40" \
 "200 r4h_lead_max1.log python scripts/host_lead.py --steps 40 --max_lead 1"

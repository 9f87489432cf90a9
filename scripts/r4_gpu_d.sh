#!/bin/bash
bash scripts/gpu_step.sh \
 "200 r4d_host_lead.log python scripts/host_lead.py --steps 20" \
 "200 r4d_host_lead_hp.log python scripts/host_lead.py --steps 20 --hp"

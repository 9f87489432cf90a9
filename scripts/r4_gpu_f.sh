#!/bin/bash
bash scripts/gpu_step.sh "300 r4f_host_ops.log python scripts/host_ops.py --steps 4 --top 40"

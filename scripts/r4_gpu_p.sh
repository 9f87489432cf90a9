#!/bin/bash
bash scripts/gpu_step.sh \
 "900 r4p_gputests.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread"

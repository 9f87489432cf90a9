#!/bin/bash
# round 5, lease p: host cost per runtime operation; host profile incl. the backward thread
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "120 r5p_launch_probe.log python scripts/launch_probe.py" \
 "300 r5p_tests.log $T tests/test_update_fused_gpu.py" \
 "200 r5p_host_cprofile.log python scripts/host_lead.py --steps 10 --hp --cprofile 10"

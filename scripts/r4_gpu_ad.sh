#!/bin/bash
bash scripts/gpu_step.sh \
 "900 r4ad_gputests.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "300 r4ad_smoke.log python -c 'import __graft_entry__ as g; g.smoke()'" \
 "150 r4ad_bench.json python bench.py"

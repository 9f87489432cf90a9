#!/bin/bash
bash scripts/gpu_step.sh \
 "900 r4f3_gputests.log python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread" \
 "300 r4f3_smoke.log python -c 'import __graft_entry__ as g; g.smoke()'" \
 "150 r4f3_bench.json python bench.py"

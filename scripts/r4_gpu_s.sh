#!/bin/bash
bash scripts/gpu_step.sh \
 "900 r4s_gputests.log python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread" \
 "300 r4s_smoke.log python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "150 r4s_bench_default.json python bench.py"

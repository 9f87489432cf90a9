#!/bin/bash
# round 5, final check of the end-of-round tree: full GPU suite, smoke, config #2
T="python -u -m pytest tests -m gpu -q -rf --tb=short --timeout 200 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "900 r5g3_gputests.log $T" \
 "300 r5g3_smoke.log python -c 'import __graft_entry__ as g; g.smoke()'" \
 "200 r5g3_bench.json python bench.py"

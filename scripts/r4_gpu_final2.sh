#!/bin/bash
bash scripts/gpu_step.sh \
 "900 r4f2_gputests.log python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread" \
 "300 r4f2_smoke.log python -c 'import __graft_entry__ as g; g.smoke()'" \
 "150 r4f2_bench.json python bench.py" \
 "150 r4f2_bench40.json python bench.py --steps 40" \
 "200 r4f2_bench_fp32.json python bench.py --fp32 --steps 20" \
 "200 r4f2_bench_fp16.json python bench.py --amp_dtype fp16 --steps 30"

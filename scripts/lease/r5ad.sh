#!/bin/bash
# round 5, lease ad: fewer weight-gradient workgroups beside the encoder backward
bash scripts/gpu_step.sh \
 "200 r5ad_div1.json python bench.py" \
 "200 r5ad_div2.json env RAFT_WGRAD_DIV=2 python bench.py" \
 "200 r5ad_div3.json env RAFT_WGRAD_DIV=3 python bench.py" \
 "200 r5ad_div1b.json python bench.py" \
 "200 r5ad_div2b.json env RAFT_WGRAD_DIV=2 python bench.py" \
 "200 r5ad_div3b.json env RAFT_WGRAD_DIV=3 python bench.py" \
 "200 r5ad_timing_div2.log env RAFT_WGRAD_DIV=2 python scripts/host_lead.py --steps 20 --hp --wgrad_timing"

#!/bin/bash
bash scripts/gpu_step.sh \
 "200 r4ah_s_new1.json python bench.py --steps 20 --batch 6 --image_size 368 768" \
 "200 r4ah_s_old1.json env RAFT_FWD6_16=0 python bench.py --steps 20 --batch 6 --image_size 368 768" \
 "150 r4ah_c2_new1.json python bench.py --steps 40" \
 "150 r4ah_c2_old1.json env RAFT_FWD6_16=0 python bench.py --steps 40" \
 "200 r4ah_s_new2.json python bench.py --steps 20 --batch 6 --image_size 368 768" \
 "200 r4ah_s_old2.json env RAFT_FWD6_16=0 python bench.py --steps 20 --batch 6 --image_size 368 768" \
 "150 r4ah_c2_new2.json python bench.py --steps 40" \
 "150 r4ah_c2_old2.json env RAFT_FWD6_16=0 python bench.py --steps 40"

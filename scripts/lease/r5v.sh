#!/bin/bash
# round 5, lease v: 1080p A/B of the round's late switches (same box, interleaved)
I="python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3"
bash scripts/gpu_step.sh \
 "200 r5v_1080_base.json $I" \
 "200 r5v_1080_rowswz.json env RAFT_SWZ_COL=0 $I" \
 "200 r5v_1080_corrv2.json env RAFT_CORR_V3=0 $I" \
 "200 r5v_1080_pystep.json env RAFT_NATIVE_STEP=0 $I" \
 "200 r5v_1080_base2.json $I" \
 "200 r5v_1080_rowswz2.json env RAFT_SWZ_COL=0 $I" \
 "200 r5v_1080_corrv22.json env RAFT_CORR_V3=0 $I" \
 "200 r5v_1080_pystep2.json env RAFT_NATIVE_STEP=0 $I" \
 "200 r5v_train_base.json python bench.py" \
 "200 r5v_train_rowswz.json env RAFT_SWZ_COL=0 python bench.py" \
 "200 r5v_train_base2.json python bench.py" \
 "200 r5v_train_rowswz2.json env RAFT_SWZ_COL=0 python bench.py"

#!/bin/bash
# Standard schedule (reference train_standard.sh), one process per GPU over RCCL.
# --batch_size is the global batch; NGPU defaults to 2 as in the reference.
# PRECISION=fp32 (default) is the reference's recipe (train_standard.sh:3-6 trains without
# --mixed_precision); PRECISION=bf16 adds bf16 autocast (train_mixed.sh keeps the reference's
# single-GPU AMP schedule).  Synthetic-data evidence of both: profiles/r3_convergence3k_*.jsonl.
NGPU=${NGPU:-2}
PRECISION=${PRECISION:-fp32}
AMP=""
if [ "$PRECISION" = "bf16" ]; then AMP="--mixed_precision"; fi
RUN="torchrun --standalone --nproc-per-node ${NGPU} --master-addr 127.0.0.1 train.py"
mkdir -p checkpoints
$RUN --name raft-chairs --stage chairs --validation chairs --num_steps 100000 --batch_size 10 --lr 0.0004 --image_size 368 496 --wdecay 0.0001 $AMP
$RUN --name raft-things --stage things --validation sintel --restore_ckpt checkpoints/raft-chairs.pth --num_steps 100000 --batch_size 6 --lr 0.000125 --image_size 400 720 --wdecay 0.0001 $AMP
$RUN --name raft-sintel --stage sintel --validation sintel --restore_ckpt checkpoints/raft-things.pth --num_steps 100000 --batch_size 6 --lr 0.000125 --image_size 368 768 --wdecay 0.00001 --gamma=0.85 $AMP
$RUN --name raft-kitti  --stage kitti --validation kitti --restore_ckpt checkpoints/raft-sintel.pth --num_steps 50000 --batch_size 6 --lr 0.0001 --image_size 288 960 --wdecay 0.00001 --gamma=0.85 $AMP

#!/bin/bash
# The current GPU session plan (one gpurun call): steps run in order by scripts/gpu_step.sh,
# each "<timeout s> <log under gpurun_out/> <command>"; the first crash / time-out ends it.
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
I1080="python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3"
TR="python train.py --stage synthetic --batch_size 1 --image_size 368 768 --num_steps 300 --iters 12 --num_workers 0 --mixed_precision --gpus 0 --ckpt_dir /tmp/ck --log_dir /tmp/runs"
bash scripts/gpu_step.sh \
 "300 r6h_train_b1_eager.log $TR --name e" \
 "300 r6h_train_b1_graph.log $TR --name g --graph" \
 "300 r6h_train_b2_eager.log $TR --name e2 --batch_size 2" \
 "300 r6h_train_b2_graph.log $TR --name g2 --batch_size 2 --graph"

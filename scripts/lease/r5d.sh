#!/bin/bash
# round 5, lease d: step profiles after the conv tiles + trainer-path throughput (device synthetic stage)
S="python scripts/rocpd_summary.py"
C="python scripts/rocpd_concurrency.py"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "400 r5d_train_synth.log python -u train.py --name r5dsynth --stage synthetic --mixed_precision --batch_size 8 --image_size 368 496 --num_steps 600 --gpus 0 --ckpt_dir gpurun_out/ckpt --log_dir gpurun_out/runs" \
 "300 r5d_prof_bf16.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r5d_bf16_kernels.txt $S gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 60" \
 "120 r5d_bf16_concurrency.txt $C gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 30 --gaps 40" \
 "30 r5d_rm.log rm -rf gpurun_out/pk" \
 "300 r5d_prof_1080.log rocprofv3 --kernel-trace -d gpurun_out/p1 -o run -- python3 bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 3 --warmup 2" \
 "120 r5d_1080_kernels.txt $S gpurun_out/p1/run_results.db --boundary corr_volume --steps 3 --top 40" \
 "30 r5d_rm2.log rm -rf gpurun_out/p1"

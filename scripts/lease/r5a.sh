#!/bin/bash
# round 5, lease a: baseline bench, trainer-path throughput, --alternate_corr kernel trace + PMC
S="python scripts/rocpd_summary.py"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "200 r5a_bench.json python bench.py" \
 "400 r5a_train_synth.log python -u train.py --name r5synth --stage synthetic --mixed_precision --batch_size 8 --image_size 368 496 --num_steps 400 --gpus 0 --ckpt_dir gpurun_out/ckpt --log_dir gpurun_out/runs" \
 "200 r5a_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "300 r5a_prof_alt.log rocprofv3 --kernel-trace -d gpurun_out/pa -o run -- python3 bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 4 --warmup 3" \
 "120 r5a_alt_kernels.txt $S gpurun_out/pa/run_results.db --boundary seq_loss_fwd --steps 3 --top 40" \
 "30 r5a_rm.log rm -rf gpurun_out/pa" \
 "400 r5a_pmc_alt.log env PMC_OUT=gpurun_out/pmc_alt PMC_CMD='bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 2 --warmup 1' bash scripts/pmc_step.sh"

#!/bin/bash
# round-4 GPU session B: correctness of the fp32 / fp16 / small paths, DDP readiness, A/Bs, traces
# (trace databases are summarised on the box and deleted: gpurun_out/ must stay under 64 MiB)
S="python scripts/rocpd_summary.py"
C="python scripts/rocpd_concurrency.py"
bash scripts/gpu_step.sh \
 "500 r4b_tests.log python -u -m pytest tests/test_split_train_gpu.py tests/test_fp16_gpu.py tests/test_golden_gpu.py -v -s --timeout 180 --timeout-method thread" \
 "300 r4b_ddp.log python -u -m pytest tests/test_ddp_gpu.py -v -s -k nccl --timeout 300 --timeout-method thread" \
 "150 r4b_bench_a1.json python bench.py --steps 30" \
 "150 r4b_bench_hp1.json env RAFT_HP_MAIN=1 python bench.py --steps 30" \
 "150 r4b_bench_a2.json python bench.py --steps 30" \
 "150 r4b_bench_hp2.json env RAFT_HP_MAIN=1 python bench.py --steps 30" \
 "200 r4b_bench_fp32_sintel.json python bench.py --fp32 --batch 6 --image_size 368 768 --steps 8 --warmup 3" \
 "200 r4b_bench_infer1080.json python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3" \
 "200 r4b_bench_small_fp32_infer.json python bench.py --small --fp32 --mode infer --image_size 440 1024 --iters 20 --batch 1 --steps 20 --warmup 3" \
 "300 r4b_prof_bf16.log rocprofv3 --kernel-trace --stats -d gpurun_out/pb -o run -- python3 bench.py --steps 4 --warmup 3" \
 "120 r4b_bf16_kernels.txt $S gpurun_out/pb/run_results.db --boundary seq_loss_fwd --steps 3 --top 60" \
 "120 r4b_bf16_concurrency.txt $C gpurun_out/pb/run_results.db --boundary seq_loss_fwd --steps 3 --top 30" \
 "30 r4b_rm1.log rm -rf gpurun_out/pb" \
 "300 r4b_prof_small_fp32_infer.log rocprofv3 --kernel-trace --stats -d gpurun_out/ps -o run -- python3 bench.py --small --fp32 --mode infer --image_size 440 1024 --iters 20 --batch 1 --steps 3 --warmup 1" \
 "120 r4b_small_fp32_infer_kernels.txt $S gpurun_out/ps/run_results.db --top 80" \
 "30 r4b_rm2.log rm -rf gpurun_out/ps" \
 "300 r4b_prof_fp16_train.log rocprofv3 --kernel-trace --stats -d gpurun_out/ph -o run -- python3 bench.py --amp_dtype fp16 --steps 4 --warmup 2" \
 "120 r4b_fp16_kernels.txt $S gpurun_out/ph/run_results.db --boundary seq_loss_fwd --steps 3 --top 80" \
 "30 r4b_rm3.log rm -rf gpurun_out/ph" \
 "300 r4b_prof_fp32_train.log rocprofv3 --kernel-trace --stats -d gpurun_out/pf -o run -- python3 bench.py --fp32 --steps 4 --warmup 2" \
 "120 r4b_fp32_kernels.txt $S gpurun_out/pf/run_results.db --boundary seq_loss_fwd --steps 3 --top 80" \
 "120 r4b_fp32_concurrency.txt $C gpurun_out/pf/run_results.db --boundary seq_loss_fwd --steps 3 --top 30" \
 "30 r4b_rm4.log rm -rf gpurun_out/pf"

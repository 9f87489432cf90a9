#!/bin/bash
S="python scripts/rocpd_summary.py"
bash scripts/gpu_step.sh \
 "200 r4n_wgrad_blas.log python scripts/bench_wgrad_blas.py" \
 "300 r4n_prof_1080.log rocprofv3 --kernel-trace -d gpurun_out/p1 -o run -- python3 bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 3 --warmup 2" \
 "120 r4n_1080_kernels.txt $S gpurun_out/p1/run_results.db --boundary corr_volume --steps 3 --top 40" \
 "30 r4n_rm.log rm -rf gpurun_out/p1" \
 "150 r4n_bench_a.json python bench.py --steps 30" \
 "150 r4n_bench_mt2.json env RAFT_WGRAD3_MT=2 python bench.py --steps 30" \
 "150 r4n_bench_a2.json python bench.py --steps 30" \
 "150 r4n_bench_mt2b.json env RAFT_WGRAD3_MT=2 python bench.py --steps 30" \
 "150 r4n_bench_a3.json python bench.py --steps 30" \
 "150 r4n_bench_mt2c.json env RAFT_WGRAD3_MT=2 python bench.py --steps 30" \
 "900 r4n_pmc.log bash scripts/pmc_step.sh"

#!/bin/bash
S="python scripts/rocpd_summary.py"
bash scripts/gpu_step.sh \
 "900 r4o_gputests.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "150 r4o_bench_a.json python bench.py --steps 30" \
 "200 r4o_bench_fp32.json python bench.py --fp32 --steps 10" \
 "300 r4o_prof_1080.log rocprofv3 --kernel-trace -d gpurun_out/p1 -o run -- python3 bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 3 --warmup 2" \
 "120 r4o_1080_grid.txt $S gpurun_out/p1/run_results.db --boundary corr_volume --steps 3 --top 40 --by-grid" \
 "30 r4o_rm.log rm -rf gpurun_out/p1" \
 "240 r4o_pmc.log env PMC_GROUPS='SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE' bash scripts/pmc_step.sh"

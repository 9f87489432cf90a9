#!/bin/bash
# round 5, lease i: alt-corr fill fix; graph-replay concurrency vs eager; host issue time
S="python scripts/rocpd_summary.py"
C="python scripts/rocpd_concurrency.py"
T="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "300 r5i_tests.log $T tests/test_kernels_gpu.py -k 'local_corr or deterministic'" \
 "200 r5i_bench_alt.json python bench.py --alternate_corr --batch 3 --image_size 376 1248 --steps 15" \
 "200 r5i_host_lead.log python scripts/host_lead.py --steps 20 --hp" \
 "300 r5i_prof_graph.log rocprofv3 --kernel-trace -d gpurun_out/pg -o run -- python3 bench.py --graph --steps 4 --warmup 3" \
 "120 r5i_graph_kernels.txt $S gpurun_out/pg/run_results.db --boundary seq_loss_fwd --steps 3 --top 20" \
 "120 r5i_graph_concurrency.txt $C gpurun_out/pg/run_results.db --boundary seq_loss_fwd --steps 3 --top 20 --gaps 30" \
 "30 r5i_rm.log rm -rf gpurun_out/pg"

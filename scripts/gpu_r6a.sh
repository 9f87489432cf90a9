export TMPDIR=/tmp
bash scripts/gpu_step.sh \
 "200 r6a_bench.json python bench.py" \
 "200 r6a_b1_368x768.json python bench.py --batch 1 --image_size 368 768" \
 "200 r6a_b2_368x768.json python bench.py --batch 2 --image_size 368 768" \
 "200 r6a_b6_368x768.json python bench.py --batch 6 --image_size 368 768" \
 "200 r6a_b1_400x720.json python bench.py --batch 1 --image_size 400 720" \
 "200 r6a_b2_400x720.json python bench.py --batch 2 --image_size 400 720" \
 "300 r6a_prof.log rocprofv3 --kernel-trace -d gpurun_out/pk -o run -- python3 bench.py --steps 4 --warmup 3 --batch 1 --image_size 368 768" \
 "120 r6a_b1_kernels.txt python scripts/rocpd_summary.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 60" \
 "120 r6a_b1_grid.txt python scripts/rocpd_summary.py gpurun_out/pk/run_results.db --boundary seq_loss_fwd --steps 3 --top 40 --by-grid" \
 "30 r6a_rm.log rm -rf gpurun_out/pk"

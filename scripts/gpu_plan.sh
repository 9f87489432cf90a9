set -o pipefail
mkdir -p gpurun_out/f
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encoder_gpu.py tests/test_golden_gpu.py tests/test_update_fused_gpu.py tests/test_train_graph.py tests/test_split_train_gpu.py > gpurun_out/f/tests.log 2>&1 || { tail -30 gpurun_out/f/tests.log; exit 1; }
tail -1 gpurun_out/f/tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f/prof_b8 -o run -- python3 bench.py --steps 6 --warmup 4 > gpurun_out/f/prof_b8.log 2>&1 || exit 1
python scripts/kernel_summary.py gpurun_out/f/prof_b8/run_kernel_trace.csv --skip 4 > gpurun_out/f/b8_kernels.txt 2>&1
head -1 gpurun_out/f/b8_kernels.txt; grep -c Fill gpurun_out/f/b8_kernels.txt || true
for r in a b; do
$T 300 python -u bench.py --steps 30 --warmup 5 > gpurun_out/f/b8_$r.json 2>/dev/null && grep -o '"value": [0-9.]*' gpurun_out/f/b8_$r.json
$T 300 python -u bench.py --steps 60 --warmup 10 --batch 1 --image_size 368 768 > gpurun_out/f/b1_$r.json 2>/dev/null && grep -o '"value": [0-9.]*' gpurun_out/f/b1_$r.json
done

set -o pipefail
mkdir -p gpurun_out/c8
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_golden_gpu.py tests/test_update_fused_gpu.py > gpurun_out/c8/tests.log 2>&1 || { tail -30 gpurun_out/c8/tests.log; exit 1; }
tail -1 gpurun_out/c8/tests.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$T 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c8/prof_b8 -o run -- python3 bench.py --steps 6 --warmup 4 > gpurun_out/c8/prof_b8.log 2>&1 || exit 1
python scripts/kernel_summary.py gpurun_out/c8/prof_b8/run_kernel_trace.csv --skip 4 > gpurun_out/c8/b8_kernels.txt 2>&1
head -1 gpurun_out/c8/b8_kernels.txt; grep -E "cin8|conv_fwd7|conv_fwd6_kernel<64, 64, 2, 2, 3, 3" gpurun_out/c8/b8_kernels.txt | cut -c1-120
for r in a b; do
$T 300 python -u bench.py --steps 30 --warmup 5 > gpurun_out/c8/b8_$r.json 2>/dev/null && grep -o '"value": [0-9.]*' gpurun_out/c8/b8_$r.json
done

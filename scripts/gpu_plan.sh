set -o pipefail
mkdir -p gpurun_out/fb
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_update_fused_gpu.py tests/test_golden_gpu.py tests/test_train_graph.py tests/test_split_train_gpu.py tests/test_model_gpu.py > gpurun_out/fb/tests.log 2>&1 || { tail -30 gpurun_out/fb/tests.log; exit 1; }
tail -1 gpurun_out/fb/tests.log
$T 300 python -u scripts/host_lead.py --batch 1 --image_size 368 768 --steps 30 --cprofile 20 > gpurun_out/fb/host_b1.log 2>&1 && grep -E "wall|forward|backward|fused_step_fwd}|update_fused.py.*forward" gpurun_out/fb/host_b1.log | head -8
for r in a b; do
$T 300 python -u bench.py --steps 30 --warmup 5 > gpurun_out/fb/b8_$r.json 2>/dev/null && grep -o '"value": [0-9.]*' gpurun_out/fb/b8_$r.json
$T 300 python -u bench.py --batch 1 --image_size 368 768 --steps 100 --warmup 10 > gpurun_out/fb/b1_$r.json 2>/dev/null && grep -o '"value": [0-9.]*' gpurun_out/fb/b1_$r.json
done

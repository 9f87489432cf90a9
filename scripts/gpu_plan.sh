set -o pipefail
mkdir -p gpurun_out/ref
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u bench.py --impl reference --steps 10 --warmup 3 > gpurun_out/ref/reference_b8.json 2> gpurun_out/ref/reference_b8.err && grep -o '"value": [0-9.]*' gpurun_out/ref/reference_b8.json
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > gpurun_out/ref/native_b8.json 2>/dev/null && grep -o '"value": [0-9.]*' gpurun_out/ref/native_b8.json

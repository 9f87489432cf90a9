set -o pipefail
mkdir -p gpurun_out/f32
export PYTHONUNBUFFERED=1
for r in a b; do
for v in 1 0; do
timeout -k 10 300 env RAFT_ENC_SPLIT3=$v python -u bench.py --fp32 --steps 10 --warmup 3 > gpurun_out/f32/split3_${v}_$r.json 2>/dev/null && echo "split3=$v $(grep -o '"value": [0-9.]*' gpurun_out/f32/split3_${v}_$r.json)"
done
done

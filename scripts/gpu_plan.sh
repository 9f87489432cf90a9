set -o pipefail
mkdir -p gpurun_out/conv
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u scripts/convergence.py --impl native --steps 3000 > gpurun_out/conv/native_bf16.jsonl 2> gpurun_out/conv/native_bf16.err || { tail -5 gpurun_out/conv/native_bf16.err; exit 1; }
tail -2 gpurun_out/conv/native_bf16.jsonl

# round-6 plan: 64 x 64 conv tiles -- correctness, then interleaved A/B of RAFT_FWD6_SMALL
set -o pipefail
mkdir -p gpurun_out/u
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_update_fused_gpu.py tests/test_golden_gpu.py > gpurun_out/u/tests.log 2>&1 || { tail -30 gpurun_out/u/tests.log; exit 1; }
tail -2 gpurun_out/u/tests.log
run() {  # tag env bench-args
  tag=$1; shift; e=$1; shift
  env $e $T 300 python -u bench.py "$@" > gpurun_out/u/$tag.json 2> gpurun_out/u/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/u/$tag.err; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/u/$tag.json)"
}
for r in a b; do
  run b8_new_$r RAFT_FWD6_SMALL=1 --steps 30 --warmup 5
  run b8_old_$r RAFT_FWD6_SMALL=0 --steps 30 --warmup 5
  run b1_new_$r RAFT_FWD6_SMALL=1 --steps 40 --warmup 5 --batch 1 --image_size 368 768
  run b1_old_$r RAFT_FWD6_SMALL=0 --steps 40 --warmup 5 --batch 1 --image_size 368 768
  run b2_new_$r RAFT_FWD6_SMALL=1 --steps 40 --warmup 5 --batch 2 --image_size 368 768
  run b2_old_$r RAFT_FWD6_SMALL=0 --steps 40 --warmup 5 --batch 2 --image_size 368 768
done
run b1t_new RAFT_FWD6_SMALL=1 --steps 40 --warmup 5 --batch 1 --image_size 400 720
run b1t_old RAFT_FWD6_SMALL=0 --steps 40 --warmup 5 --batch 1 --image_size 400 720
run inf1080_new RAFT_FWD6_SMALL=1 --mode infer --batch 1 --image_size 1080 1920 --iters 32 --steps 20 --warmup 5
run inf1080_old RAFT_FWD6_SMALL=0 --mode infer --batch 1 --image_size 1080 1920 --iters 32 --steps 20 --warmup 5

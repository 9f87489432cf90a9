# round-6 plan: native backward step executor -- allocator check, then interleaved A/B of RAFT_NATIVE_BWD
set -o pipefail
mkdir -p gpurun_out/w
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 300 python -u scripts/host_lead.py --batch 1 --image_size 368 768 --steps 30 > gpurun_out/w/host_lead_b1.log 2>&1 && tail -12 gpurun_out/w/host_lead_b1.log || exit 1
run() {  # tag env bench-args
  tag=$1; shift; e=$1; shift
  env $e $T 300 python -u bench.py "$@" > gpurun_out/w/$tag.json 2> gpurun_out/w/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/w/$tag.err; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/w/$tag.json) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/w/$tag.json)"
}
for r in a b c; do
  run b1_new_$r RAFT_NATIVE_BWD=1 --steps 200 --warmup 20 --batch 1 --image_size 368 768
  run b1_old_$r RAFT_NATIVE_BWD=0 --steps 200 --warmup 20 --batch 1 --image_size 368 768
  run b2_new_$r RAFT_NATIVE_BWD=1 --steps 100 --warmup 20 --batch 2 --image_size 368 768
  run b2_old_$r RAFT_NATIVE_BWD=0 --steps 100 --warmup 20 --batch 2 --image_size 368 768
done

#!/bin/bash
# One GPU-box session of measurements (each step has its own time limit; any abnormal exit
# -- crash, abort, timeout -- ends the script).  Outputs land in gpurun_out/measure/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/measure
mkdir -p $OUT
export TMPDIR=/tmp

run() {  # run <name> <timeout-seconds> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "    rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}

for step in ${STEPS_LIST:-infer1080 infer_sintel alt_kitti dense_kitti conv_native conv_reference}; do
  case $step in
    infer1080) run infer1080 300 python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3 ;;
    infer_sintel) run infer_sintel 300 python bench.py --mode infer --image_size 440 1024 --iters 32 --batch 1 --steps 20 --warmup 3 ;;
    alt_kitti) run alt_kitti 300 python bench.py --alternate_corr --image_size 376 1248 --batch 3 --steps 10 --warmup 3 ;;
    dense_kitti) run dense_kitti 300 python bench.py --image_size 376 1248 --batch 3 --steps 10 --warmup 3 ;;
    conv_native) run conv_native 600 python scripts/convergence.py --impl native --steps ${CONV_STEPS:-2000} ;;
    conv_reference) run conv_reference 900 python scripts/convergence.py --impl reference --steps ${CONV_STEPS:-2000} ;;
    conv_fp32) run conv_fp32 1100 python scripts/convergence.py --impl native --precision fp32 --steps ${CONV_STEPS:-3000} --eval_every 250 ;;
    conv_bf16) run conv_bf16 600 python scripts/convergence.py --impl native --precision bf16 --steps ${CONV_STEPS:-3000} --eval_every 250 ;;
    ref_bench) run ref_bench 600 python bench.py --impl reference --steps 10 --warmup 3 ;;
    train) run train 300 python bench.py --steps 30 --warmup 5 ;;
    train_graph) run train_graph 300 python bench.py --graph --steps 30 --warmup 5 ;;
    infer1080_eager) run infer1080_eager 300 python bench.py --mode infer --no-graph --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3 ;;
    train_fp32) run train_fp32 400 python bench.py --fp32 --steps 10 --warmup 3 ;;
    infer_ros_fp32) run infer_ros_fp32 300 python bench.py --mode infer --fp32 --image_size 440 1024 --iters 20 --batch 1 --steps 20 --warmup 3 ;;
    infer_ros_bf16) run infer_ros_bf16 300 python bench.py --mode infer --image_size 440 1024 --iters 20 --batch 1 --steps 20 --warmup 3 ;;
    alt_ros_fp32) run alt_ros_fp32 300 python bench.py --mode infer --fp32 --alternate_corr --image_size 440 1024 --iters 20 --batch 1 --steps 20 --warmup 3 ;;
    train_sintel) run train_sintel 300 python bench.py --image_size 368 768 --batch 6 --steps 20 --warmup 5 ;;
    train_full) run train_full 300 python bench.py --image_size 440 1024 --batch 6 --steps 10 --warmup 3 ;;
    prof_fp32) run prof_fp32 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp32 -o run -- python3 bench.py --mode infer --fp32 --image_size 440 1024 --iters 20 --batch 1 --steps 5 --warmup 2 ;;
    prof_train) run prof_train 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_train -o run -- python3 bench.py --steps 8 --warmup 4 ;;
    prof_infer1080) run prof_infer1080 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_infer1080 -o run -- python3 bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 5 --warmup 2 ;;
  esac
done
echo done

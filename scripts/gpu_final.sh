#!/bin/bash
# Round-end validation: full GPU suite, smoke, training bench, inference benches (configs #5
# and Sintel), each step under its own time limit; stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
run() {  # run <name> <timeout-seconds> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "    rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --tb=short --timeout 200 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_train 300 python bench.py --steps 30 --warmup 5
run bench_infer1080 300 python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3
run bench_infer_sintel 300 python bench.py --mode infer --image_size 440 1024 --iters 32 --batch 1 --steps 20 --warmup 3
echo done

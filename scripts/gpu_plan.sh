#!/bin/bash
# Round-6 end-of-round check on the final tree: full GPU suite, smoke, config #2 and batch-1 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/end
mkdir -p $OUT
export PYTHONUNBUFFERED=1
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $OUT/$name.log | head -1) $(tail -n 1 $OUT/$name.log | cut -c1-100)"
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --tb=short --timeout 200 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step b8_a 300 python bench.py --steps 30 --warmup 5
step b8_b 300 python bench.py --steps 30 --warmup 5
step b1 300 python bench.py --batch 1 --image_size 368 768 --steps 100 --warmup 10
step b6 300 python bench.py --batch 6 --image_size 368 768 --steps 20 --warmup 5
step infer1080 300 python bench.py --mode infer --image_size 1080 1920 --iters 32 --batch 1 --steps 10 --warmup 3
echo done

#!/bin/bash
# One GPU-box session: GPU tests, smoke, benches and a rocprofv3 kernel profile.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script
# (exit codes 0/1 = ran to completion, anything else = stop).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp

run() {  # run <name> <timeout-seconds> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "    rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}

STEPS=${STEPS:-10}
run pytest_gpu 900 python -m pytest tests -m gpu -x -q
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_native 600 python bench.py --steps "$STEPS" --warmup 3
if [ "${SKIP_REF:-0}" != "1" ]; then
  run bench_reference 900 python bench.py --steps "$STEPS" --warmup 3 --impl reference
fi
if [ "${PROFILE:-1}" = "1" ]; then
  run rocprof_native 900 rocprofv3 --kernel-trace --stats -d $OUT/prof_native -o run -- python3 bench.py --steps 3 --warmup 2
fi
echo "done"

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
if [ "${TESTS:-1}" = "1" ]; then
  run pytest_gpu 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -q -rf --tb=short --timeout 200 --timeout-method thread ${PYTEST_ARGS:-}
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "${BENCH:-1}" = "1" ]; then
  run bench_native 600 python bench.py --steps "$STEPS" --warmup 3 ${BENCH_ARGS:-}
fi
if [ "${SKIP_REF:-1}" != "1" ]; then
  run bench_reference 900 python bench.py --steps "$STEPS" --warmup 3 --impl reference
fi
if [ "${PROFILE:-1}" = "1" ]; then
  TAG=${TAG:-native}
  run rocprof_$TAG 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- python3 bench.py --steps 4 --warmup 3 ${PROF_ARGS:-}
  python scripts/kernel_summary.py $OUT/prof_$TAG/run_kernel_trace.csv --boundary "${BOUNDARY:-seq_loss_fwd}" --every "${EVERY:-1}" --skip 3 --out $OUT/prof_$TAG/steady_summary.csv > $OUT/prof_$TAG/steady_summary.txt 2>&1
  KPS=$(head -1 $OUT/prof_$TAG/steady_summary.txt | sed -n 's/.*kernels\/step=\([0-9]*\).*/\1/p')
  [ -n "$KPS" ] && python scripts/kernel_timeline.py $OUT/prof_$TAG/run_kernel_trace.csv --per-step "$KPS" --list > $OUT/prof_$TAG/steady_timeline.txt 2>&1
  python scripts/kernel_shapes.py $OUT/prof_$TAG/run_kernel_trace.csv --steps 4 --top 60 > $OUT/prof_$TAG/steady_shapes.txt 2>&1
  # keep only the summaries (the per-dispatch trace is too large to ship back)
  find $OUT/prof_$TAG -type f ! -name '*stats*' ! -name 'steady_*' -delete
fi
echo "done"

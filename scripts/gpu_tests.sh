#!/bin/bash
# GPU test pass: selected test files (default: all) under one time limit, then smoke.
# usage: bash scripts/gpu_tests.sh [pytest args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
[ $# -eq 0 ] && set -- tests
timeout -k 10 ${TEST_LIMIT:-500} python -u -m pytest "$@" -m gpu -x -v -s --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|EPE|rel|delta" gpurun_out/pytest_gpu.log | tail -40
tail -3 gpurun_out/pytest_gpu.log
exit $rc

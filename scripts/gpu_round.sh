#!/bin/bash
# One GPU pass: tests (train-graph test last), smoke, 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  --deselect tests/test_train_graph.py::test_graphed_step_replay_matches_eager_gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 200 python -u -m pytest tests/test_train_graph.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tg.log 2>&1; echo "train-graph rc=$?"; grep -E "passed|failed|Error" gpurun_out/tg.log | tail -3

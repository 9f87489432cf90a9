#!/bin/bash
# Round-3 evidence run: kernel-trace profile of the training step and of 1080p inference,
# PMC counters of the training step (one counter group per rocprofv3 pass), and the
# config #3 / #4 shape benches.  Each step under its own time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_update_fused_gpu.py > gpurun_out/t_evidence.log 2>&1 || { tail -20 gpurun_out/t_evidence.log; exit 1; }
tail -1 gpurun_out/t_evidence.log
STEPS_LIST="prof_train prof_infer1080 train_sintel train_full alt_kitti dense_kitti" bash scripts/gpu_measure.sh || exit $?
find gpurun_out/measure -name "*.csv" -size +20M -delete
PMC_OUT=gpurun_out/pmc_step bash scripts/pmc_step.sh || exit $?
echo evidence-done

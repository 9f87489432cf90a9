#!/bin/bash
# Run GPU steps in order; stop at the first step that crashes / times out (rc not in {0, 1}).
# usage: bash scripts/gpu_step.sh "<timeout> <logname> <cmd...>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  to=${spec%% *}; rest=${spec#* }; log=${rest%% *}; cmd=${rest#* }
  echo "[gpu_step] $cmd (timeout $to) -> gpurun_out/$log"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "[gpu_step] rc=$rc"
  tail -3 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_step] stopping after rc=$rc"; exit $rc; fi
done

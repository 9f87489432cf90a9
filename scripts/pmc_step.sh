#!/bin/bash
# PMC counters of one short training step, one counter group per rocprofv3 run
# (--kernel-trace + --pmc only; no runtime/sys trace), aggregated per kernel by
# scripts/pmc_summary.py.  Usage (on the GPU box):  bash scripts/pmc_step.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_step}
mkdir -p $OUT
CMD=${PMC_CMD:-bench.py --steps 2 --warmup 1}
GROUPS_DEFAULT="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
GROUPS_DEFAULT="$GROUPS_DEFAULT;SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY"
GROUPS_DEFAULT="$GROUPS_DEFAULT;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
IFS=';' read -ra GROUP_LIST <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
i=0
for grp in "${GROUP_LIST[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/g$i -o run -- python3 $CMD > $OUT/g$i.log 2>&1
  rc=$?
  echo "group $i ($grp): rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/g$i.log; exit $rc; fi
done
python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt
find $OUT -name '*.csv' -size +1M -delete
cat $OUT/summary.txt

#!/bin/bash
# PMC counters for single conv shapes (own run, --kernel-trace only, no sys/runtime trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
IFS=, read -ra SPEC_LIST <<< "${SPECS:-zr fwd 8,zr wgrad,mask2 wgrad}"
for spec in "${SPEC_LIST[@]}"; do
  tag=$(echo $spec | tr ' ' '_')
  IFS=';' read -ra GROUP_LIST <<< "${PMC_GROUPS:-SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS;SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM;TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE}"
  for grp in "${GROUP_LIST[@]}"; do
    g=$(echo $grp | cut -d' ' -f1)
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/$tag/$g -o run -- python3 scripts/conv_one.py $spec > $OUT/$tag.$g.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag $g rc=$rc"; tail -3 $OUT/$tag.$g.log; fi
    if [ $rc -gt 1 ]; then exit $rc; fi
  done
done
python3 - <<'PY'
import csv, glob, collections, os
res = collections.defaultdict(dict)
for f in glob.glob(os.environ.get('PMC_OUT', 'gpurun_out/pmc') + '/*/*/run_counter_collection.csv'):
    tag = f.split('/')[-3]
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(list)
    for r in rows:
        if 'raft_amd' not in r['Kernel_Name']: continue
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in agg.items():
        v.sort(); res[tag][k] = v[len(v)//2]
with open(os.environ.get('PMC_OUT', 'gpurun_out/pmc') + '/summary.txt', 'w') as fo:
    for tag in sorted(res):
        fo.write(tag + ': ' + ', '.join(f"{k}={v:.4g}" for k, v in sorted(res[tag].items())) + '\n')
PY
find $OUT -name '*.csv' ! -name 'summary*' -size +2M -delete
cat $OUT/summary.txt

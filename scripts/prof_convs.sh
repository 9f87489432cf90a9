cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_convs
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_convs -o run -- python3 scripts/bench_convs.py --cfg 2,4,6 > gpurun_out/prof_convs/log.txt 2>&1
rc=$?
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/prof_convs/run_kernel_trace.csv')))
# group by kernel name + grid size (distinguishes shapes)
agg = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name']
    if 'raft_amd' not in n and 'igemm' not in n and 'ck' not in n and 'conv' not in n.lower(): continue
    key = (n[:90], r.get('Grid_Size', r.get('Grid_Size_X','?')))
    agg[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
with open('gpurun_out/prof_convs/per_kernel.txt', 'w') as f:
    for (n, g), v in sorted(agg.items(), key=lambda kv: kv[0]):
        v.sort()
        f.write(f"{len(v):4d} med={v[len(v)//2]:8.1f}us grid={g:>8} {n}\n")
PY
find gpurun_out/prof_convs -type f ! -name '*stats*' ! -name 'per_kernel.txt' ! -name 'log.txt' -delete
exit $rc

mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/tprof
TN_ONLY_AUTO=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tprof -o run -- python3 tools/tn_bench.py > gpurun_out/tn_prof.txt 2>&1; rc=$?
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/tprof/**/*kernel_trace.csv', recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'tn' in r['Kernel_Name'] or 'skinny' in r['Kernel_Name']:
        agg[(r['Kernel_Name'][:50], r['Grid_Size_X'], r['Workgroup_Size_X'])].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
for k, v in agg.items():
    v = sorted(v)
    print(f"{len(v):4d} median {v[len(v)//2]/1e3:7.1f} us  {k}")
PY
exit $rc

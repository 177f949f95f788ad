# per-frame call anatomy (host phases + kernel trace) and the VALU price in GRBM cycles
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5d}; mkdir -p $O
VO_PF_PROFILE=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
cat $O/pf.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/pftrace -o pf -- python3 tools/pf_loop.py 30 > $O/pftrace.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/pftrace.txt; exit 1; }
python3 tools/pf_timeline.py $O/pftrace > $O/pf_timeline.txt 2>&1; cat $O/pf_timeline.txt
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/valu -o valu -- ./tools/valu_rate > $O/valu_pmc.txt 2>&1 || { echo VALUPMC_FAIL; tail $O/valu_pmc.txt; exit 1; }
python3 - <<'PY'
import csv, glob, collections
rows = collections.defaultdict(dict)
for f in glob.glob('gpurun_out/r5d/valu/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        rows[(r['Kernel_Name'][:30], r.get('Dispatch_Id', r.get('Correlation_Id', '')))][r['Counter_Name']] = float(r['Counter_Value'])
for k, v in sorted(rows.items()):
    if 'SQ_INSTS_VALU' in v and 'GRBM_GUI_ACTIVE' in v and v['GRBM_GUI_ACTIVE'] > 0:
        print(k[0], 'VALU', int(v['SQ_INSTS_VALU']), 'GRBM', int(v['GRBM_GUI_ACTIVE']),
              'cycles per wave64 VALU per SIMD:', round(1024 * v['GRBM_GUI_ACTIVE'] / 8 / v['SQ_INSTS_VALU'], 2))
PY
echo DONE

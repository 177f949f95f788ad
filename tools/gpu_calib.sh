# FETCH_SIZE / WRITE_SIZE calibration per access width (tools/fetch_calib.hip), the counter list,
# and the config-2 extract parity test
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/calib; mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O -o fetch -- ./tools/fetch_calib > $O/fetch.log 2>&1 || { echo FETCH_FAIL; tail $O/fetch.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O -o write -- ./tools/fetch_calib > $O/write.log 2>&1 || { echo WRITE_FAIL; tail $O/write.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O -o valu -- ./tools/fetch_calib > $O/valu.log 2>&1 || { echo VALU_FAIL; tail $O/valu.log; exit 1; }
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob('gpurun_out/calib/**/*counter_collection.csv', recursive=True)):
    print(f)
    for r in csv.DictReader(open(f)):
        print(' ', r['Kernel_Name'][:40], r['Counter_Name'], r['Counter_Value'])
PY
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread -k config2 > $O/cfg2.log 2>&1 || { echo CFG2_FAIL; tail -30 $O/cfg2.log; exit 1; }
tail -2 $O/cfg2.log

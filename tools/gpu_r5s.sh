# full GPU suite on the current build; the bench's variants (live vs rocprof for the 0.12 RANSAC row)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5s}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
timeout -k 10 600 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('VALUE',round(d['value']));v=d['variants'];print(round(v['low_inlier_0.12']['fps']), v['low_inlier_0.12']['roofline']['avg_launch_ms'], v['low_inlier_0.12']['roofline']['rocprof_avg_launch_us'], v['low_inlier_0.12']['roofline']['frames_per_launch']);print(v['process_frame'])"
echo DONE

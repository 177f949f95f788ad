# round 3: new regime parity tests + knob tests + smoke + default bench (CPU leg included)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3a}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_regimes.py "tests/test_gpu_paths.py::test_process_knobs_match_oracle" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python -u bench.py --breakdown > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('VALUE',round(d['value']),'dominant',d['roofline']['kernel'], d['determinism'], d['config']['fitted_fraction'], d['h2d_inclusive']); print(json.dumps(d['variants']['low_inlier_0.12'].get('roofline'))); print(json.dumps(d['cpu_baseline'])[:600])"
cat $O/bench.err

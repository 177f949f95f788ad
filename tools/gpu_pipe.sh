# pipelined pose passes: parity (regimes, paths, parity) then A/B of VO_PIPELINE at 1.0 and 0.12 m/frame
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pipe}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_regimes.py tests/test_gpu_paths.py tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for m in 1.0 0.12; do
for rep in 1 2; do
for e in "VO_PIPELINE=0" "VO_PIPELINE=1"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --motion $m > $O/b.json 2> $O/b.err || { echo FAIL "$e"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$m', '$e', round(d['value']), d['determinism']['gathered_rows_equal_separate_runs'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
done

# parity subset (extract / match / trajectory) + 3 bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-q2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_paths.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --no-cpu --no-variants --no-check > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done

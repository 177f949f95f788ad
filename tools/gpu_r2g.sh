set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu --no-variants > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail $O/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']), {k: v['us_per_launch'] for k, v in d['kernels'].items()})"
done
timeout -k 10 300 python -u bench.py --no-cpu --no-variants --width 1920 --height 1080 --max-kpts 4096 --frames 64 --sequences 4 > $O/bx.json 2> $O/bx.err || { echo BENCHX_FAIL; tail $O/bx.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bx.json'));print('1080', round(d['value']), {k: v['us_per_launch'] for k, v in d['kernels'].items()})"

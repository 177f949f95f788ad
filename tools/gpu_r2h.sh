set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 120 python -u tools/stamps_ransac.py > $O/stamps_ransac.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_ransac.txt; exit 1; }
tail -4 $O/stamps_ransac.txt
for r in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu --no-variants > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail $O/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']), {k: v['us_per_launch'] for k, v in d['kernels'].items()})"
timeout -k 10 300 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 2 > $O/b12.json 2> $O/b12.err || { echo BENCH_FAIL; tail $O/b12.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b12.json'));print('0.12', round(d['value']), {k: v['us_per_launch'] for k, v in d['kernels'].items()})"
done
VO_SERIAL=1 timeout -k 10 300 python -u bench.py --no-cpu --no-variants --sequences 2 > $O/bs.json 2> $O/bs.err || { echo BENCH_FAIL; tail $O/bs.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bs.json'));print('serial', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"

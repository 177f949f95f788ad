set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2o; mkdir -p $O
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 120 python -u tools/stamps_finalize.py > $O/stamps_fin.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_fin.txt; exit 1; }
cat $O/stamps_fin.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu --no-variants > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail $O/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']), d['ms_per_step'])"
done

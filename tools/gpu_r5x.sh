# k_select key staging by waves: parity, stamps, KITTI A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5x}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regimes.py tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 200 python3 tools/stamps_select_batched.py > $O/sel.txt 2>&1 || { echo STAMPS_FAIL; tail $O/sel.txt; exit 1; }
cat $O/sel.txt
for rep in 1 2 3; do for lib in libvo_mi355x.so libvo_mi355x_sel0.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants > $O/b.json 2> $O/b.err || { echo "KITTI BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('KITTI $lib', round(d['value']), d['kernels']['select']['us_per_frame'])"
done; done
echo DONE

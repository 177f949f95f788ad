# describe_pf terms in three sweeps; later RANSAC chunks stop a wave's count once it cannot pass the
# best (A/B against RS_EARLY=0); parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5k}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py tests/test_gpu_regimes.py tests/test_gpu_reference_sampler.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so PF=1 timeout -k 10 200 python3 tools/stamps_describe.py > $O/stamps_describe_pf.txt 2>&1 || { echo STAMPS_DS_FAIL; tail $O/stamps_describe_pf.txt; exit 1; }
cat $O/stamps_describe_pf.txt
for e in 1 2; do
  PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "pf $(tail -1 $O/pf.txt)"
done
for rep in 1 2; do for lib in libvo_mi355x.so libvo_mi355x_early0.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/b.json 2> $O/b.err || { echo "BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('0.12 $lib', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done; done
for lib in libvo_mi355x.so libvo_mi355x_early0.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants > $O/b.json 2> $O/b.err || { echo "KITTI BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('KITTI $lib', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
echo DONE

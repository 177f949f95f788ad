# Gauss-Jordan: group pivot by max-then-min-index, pivot row through LDS (A/B against gj0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5n}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regimes.py tests/test_gpu_reference_sampler.py tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so STAGE=1 MOTION=0.12 timeout -k 10 200 python3 tools/stamps_ransac.py > $O/stamps_stage.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_stage.txt; exit 1; }
cat $O/stamps_stage.txt
for rep in 1 2; do for lib in libvo_mi355x.so libvo_mi355x_gj0.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/b.json 2> $O/b.err || { echo "BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('0.12 $lib', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done; done
for lib in libvo_mi355x.so libvo_mi355x_gj0.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "pf $lib $(tail -1 $O/pf.txt)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ktrace -o tr -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-variants > $O/ktrace.json 2>&1 || { echo TRACE_FAIL; exit 1; }
echo DONE

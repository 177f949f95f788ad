# RANSAC later chunks on the fit queue, count word assembly from lane masks, describe_pf tables in
# LDS, fused select by default: parity, per-frame latency, 0.12 / KITTI A/B of the split
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5j}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py tests/test_gpu_regimes.py tests/test_gpu_reference_sampler.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so PF=1 timeout -k 10 200 python3 tools/stamps_describe.py > $O/stamps_describe_pf.txt 2>&1 || { echo STAMPS_DS_FAIL; tail $O/stamps_describe_pf.txt; exit 1; }
cat $O/stamps_describe_pf.txt
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so STAGE=1 MOTION=0.12 timeout -k 10 200 python3 tools/stamps_ransac.py > $O/stamps_stage.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_stage.txt; exit 1; }
cat $O/stamps_stage.txt
for e in "VO_X=0" "VO_SEL_FUSED=0" "VO_X=0" "VO_SEL_FUSED=0"; do
  env $e PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$e $(tail -1 $O/pf.txt)"
done
PF_PINNED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pftrace -o pf -- python3 tools/pf_loop.py 30 > $O/pftrace.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/pftrace.txt; exit 1; }
python3 tools/pf_timeline.py $O/pftrace > $O/pf_timeline.txt 2>&1; cat $O/pf_timeline.txt
for rep in 1 2; do for e in "VO_RANSAC_SPLIT=1" "VO_RANSAC_SPLIT=0"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/b.json 2> $O/b.err || { echo "BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('0.12 $e', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done; done
for e in "VO_RANSAC_SPLIT=1" "VO_RANSAC_SPLIT=0"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants > $O/b.json 2> $O/b.err || { echo "KITTI BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('KITTI $e', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/trace.json 2>&1 || { echo TRACE_FAIL; exit 1; }
echo DONE

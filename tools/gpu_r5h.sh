# RANSAC count ILP: parity of the new count (product build), phase stamps, and an A/B of the
# register-budget variants at 0.12 m/frame (one 200-frame sequence) plus the adaptive segments
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5h}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regimes.py tests/test_gpu_reference_sampler.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so STAGE=1 MOTION=0.12 timeout -k 10 200 python3 tools/stamps_ransac.py > $O/stamps_stage.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_stage.txt; exit 1; }
cat $O/stamps_stage.txt
for rep in 1 2; do
for lib in libvo_mi355x.so libvo_mi355x_ilp0.so libvo_mi355x_j4pf0.so libvo_mi355x_j2pf0.so libvo_mi355x_pf0.so libvo_mi355x_j4pf1.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/b.json 2> $O/b.err || { echo "$lib BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('$lib', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
VO_STSEG_ADAPT=0 timeout -k 10 200 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/b.json 2> $O/b.err || { echo "ADAPT0 BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b.json')); print('STSEG_ADAPT=0', round(d['value']))"
done
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so PF=1 timeout -k 10 200 python3 tools/stamps_describe.py > $O/stamps_describe_pf.txt 2>&1 || { echo STAMPS_DS_FAIL; tail $O/stamps_describe_pf.txt; exit 1; }
cat $O/stamps_describe_pf.txt
for e in "VO_X=0" "VO_RANSAC_FUSED=0" "VO_SEL_FUSED=1" "VO_X=0" "VO_RANSAC_FUSED=0" "VO_SEL_FUSED=1"; do
  env $e PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$e $(tail -1 $O/pf.txt)"
done
echo DONE

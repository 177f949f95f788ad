# A/B of the matcher candidate-loop unroll (MT_UNROLL 4 default vs 1 / 2 builds): parity tests, then bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/mu; mkdir -p $O
for lib in libvo_mi355x_mu1.so libvo_mi355x_mu2.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/$lib.log 2>&1 || { echo "$lib PYTEST_FAIL"; tail -20 $O/$lib.log; exit 1; }
  echo "$lib $(tail -1 $O/$lib.log)"
done
for rep in 1 2; do
for lib in libvo_mi355x.so libvo_mi355x_mu1.so libvo_mi355x_mu2.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --breakdown > $O/b_$lib.json 2> $O/b_$lib.err || { echo "$lib BENCH_FAIL"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/b_$lib.json')); print('$lib kitti', round(d['value']), 'match us/launch', d['kernels_ms_per_launch']['match']*1e3)"
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --width 1920 --height 1080 --max-kpts 4096 > $O/bx_$lib.json 2> $O/bx_$lib.err || { echo "$lib BENCHX_FAIL"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bx_$lib.json')); print('$lib 1080', round(d['value']), 'match us/launch', d['kernels_ms_per_launch']['match']*1e3)"
done
done
echo DONE

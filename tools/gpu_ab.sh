# A/B of library builds (make -C acs_visual_odometry_amd/csrc variant NAME=<tag> DEFS=...):
# every -m gpu parity test per build, then two alternating bench runs per build.
#   AB_LIBS="libvo_mi355x.so libvo_mi355x_<tag>.so" bash tools/gpu_ab.sh [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
LIBS=${AB_LIBS:-libvo_mi355x.so}
for lib in $LIBS; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/$lib.log 2>&1 || { echo "$lib PYTEST_FAIL"; tail -20 $O/$lib.log; exit 1; }
  echo "$lib $(tail -1 $O/$lib.log)"
done
for rep in 1 2; do
for lib in $LIBS; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants "$@" > $O/b_$lib.json 2> $O/b_$lib.err || { echo "$lib BENCH_FAIL"; tail -5 $O/b_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$lib.json')); print('$lib', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
echo DONE

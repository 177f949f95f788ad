# bench A/B of library builds: gpu_ab_libs.sh <tag> "<lib A> <lib B> ..." [bench args] (no parity run)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O; LIBS="$2"; shift 2
for rep in 1 2 3; do
for lib in $LIBS; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants "$@" > $O/b.json 2> $O/b.err || { echo "$lib BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('$lib', '${VO_SERIAL:-}', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done

# Alternating A/B of library builds with R repetitions, bench value only (noise-resolving runs):
#   gpu_ab_reps.sh <tag> <reps> "<lib A> <lib B> ..." [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; R=$2; LIBS="$3"; shift 3; mkdir -p $O
for rep in $(seq 1 $R); do
for lib in $LIBS; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants --no-check "$@" > $O/b.json 2> $O/b.err || { echo "$lib BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('$lib', round(d['value']))"
done
done

# alternating bench lines over library builds (args: out-tag lib...), rows checked
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-ablibs}; mkdir -p $O
shift
for rep in 1 2 3; do
for lib in "$@"; do
  VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants --steps 10 > $O/b.json 2> $O/b.err || { echo FAIL "$lib"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$lib', round(d['value']), d['determinism']['timed_rows_equal_warmup_rows'], d['determinism']['gathered_rows_equal_separate_runs'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
echo DONE

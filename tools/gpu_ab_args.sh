# A/B of bench arguments, alternating: gpu_ab_args.sh <tag> "<args A>" "<args B>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O; shift
for rep in 1 2; do
for a in "$@"; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-variants --no-check $a > $O/b.json 2> $O/b.err || { echo FAIL "$a"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$a', round(d['value']), d['determinism'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done

# alternating bench lines over execution knobs (env settings separated by ';' inside one argument)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-knobs}; mkdir -p $O
shift
for rep in 1 2; do
for e in "$@"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --no-check --steps 10 > $O/b.json 2> $O/b.err || { echo FAIL "$e"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$e', round(d['value']), d['determinism']['timed_rows_equal_warmup_rows'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
echo DONE

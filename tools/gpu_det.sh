# determinism probe: the bench's row checks under execution knobs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-det}; mkdir -p $O
shift
for e in "$@"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --steps 10 > $O/b.json 2> $O/b.err || { echo FAIL "$e"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$e', round(d['value']), d['determinism']['timed_rows_equal_warmup_rows'], d['determinism']['gathered_rows_equal_separate_runs'], d['config']['fitted_fraction'])"
done
echo DONE

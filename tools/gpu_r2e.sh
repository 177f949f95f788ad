set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u bench.py --breakdown > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench.json'))
print('VALUE',round(d['value']),'dominant',d['roofline']['kernel'], d['determinism'])
v=d['variants']
print({k:(round(x['fps']), x.get('ratio')) for k,x in v.items()})
"
cat $O/bench.err

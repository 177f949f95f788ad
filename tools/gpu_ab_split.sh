# A/B of the split extract queues (VO_SPLIT): parity subset under the split, then alternating bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-split}; mkdir -p $O
VO_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do for S in 0 1; do
VO_SPLIT=$S timeout -k 10 300 python -u bench.py --no-cpu --no-variants --no-check --breakdown > $O/b_$S_$i.json 2> $O/b_${S}_$i.err || { echo BENCH_FAIL; tail -20 $O/b_${S}_$i.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b_$S_$i.json'));print('SPLIT=$S', round(d['value']))"
done; done
cat $O/b_1_2.err

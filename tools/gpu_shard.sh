# within-sequence sharding GPU parity + the quick parity subset and a bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-shard}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py -k "shard" -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_shard.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest_shard.log; exit 1; }
tail -3 $O/pytest_shard.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu --no-variants --breakdown > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('VALUE',round(d['value'],1))"
cat $O/bench.err

# full round check on the GPU box: every -m gpu test, smoke(), the default bench (with the
# CPU leg), the 1920x1080/N=4096 bench, and a kernel-trace stats profile of the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-full}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python -u bench.py --breakdown > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json; cat $O/bench.err
timeout -k 10 300 python -u bench.py --no-cpu --width 1920 --height 1080 --max-kpts 4096 > $O/bench_1080.json 2> $O/bench_1080.err || { echo BENCH1080_FAIL; tail -20 $O/bench_1080.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_1080.json'));print('1080 VALUE',round(d['value'],1))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o stats -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/prof_bench.json 2>&1 || { echo PROF_FAIL; exit 1; }
echo DONE

# quick GPU iteration: parity subset, bench (no CPU leg), kernel trace timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-q}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu --breakdown > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('VALUE',round(d['value'],1),'dominant',d['roofline']['kernel'],round(d['roofline']['avg_launch_ms']*1e3,1),'us')"
cat $O/bench.err
timeout -k 10 300 python -u bench.py --no-cpu --width 1920 --height 1080 --max-kpts 4096 > $O/bench_1080.json 2> $O/bench_1080.err || { echo BENCH1080_FAIL; tail -20 $O/bench_1080.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_1080.json'));print('1080 VALUE',round(d['value'],1))"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o trace -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/prof_bench.json 2>&1 || { echo PROF_FAIL; exit 1; }
python3 tools/timeline.py $O/prof/trace_kernel_trace.csv

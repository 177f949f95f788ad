# full GPU suite; first pass of a chunk on the fit queue (A/B), split-count latency RANSAC (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5m}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for e in "VO_RANSAC_SPLIT_COUNT=1" "VO_RANSAC_SPLIT_COUNT=0"; do
  env $e PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$e $(tail -1 $O/pf.txt)"
done; done
PF_PINNED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pftrace -o pf -- python3 tools/pf_loop.py 30 > $O/pftrace.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/pftrace.txt; exit 1; }
python3 tools/pf_timeline.py $O/pftrace > $O/pf_timeline.txt 2>&1; cat $O/pf_timeline.txt
for rep in 1 2; do for e in "VO_PIPE_FIRST=1" "VO_PIPE_FIRST=0"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/b.json 2> $O/b.err || { echo "BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('0.12 $e', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done; done
for e in "VO_PIPE_FIRST=1" "VO_PIPE_FIRST=0"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants > $O/b.json 2> $O/b.err || { echo "KITTI BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('KITTI $e', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/trace.json 2>&1 || { echo TRACE_FAIL; exit 1; }
echo DONE

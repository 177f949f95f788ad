# extract-queue gap after describe: batch events vs wait-value packets without events (A/B + trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5p}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q -k "process_knobs" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do for e in "VO_EVENT_WAIT=1" "VO_EVENT_WAIT=0" "VO_EVENT_WAIT=0 VO_EV_SKIP=1"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants > $O/b.json 2> $O/b.err || { echo "KITTI BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('KITTI $e', round(d['value']))"
done; done
VO_EVENT_WAIT=0 VO_EV_SKIP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ktrace -o tr -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-variants > $O/ktrace.json 2>&1 || { echo TRACE_FAIL; exit 1; }
echo DONE

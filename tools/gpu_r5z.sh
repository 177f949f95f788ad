# later RANSAC chunks on the trajectory queue (VO_RANSAC_Q=1): parity, 0.12 and KITTI A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5z}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q -k "queue_knobs" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_RANSAC_Q=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_regimes.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest2.log 2>&1 || { echo PYTEST2_FAIL; tail -40 $O/pytest2.log; exit 1; }
tail -1 $O/pytest2.log
for rep in 1 2 3; do for e in "VO_RANSAC_Q=1" "VO_RANSAC_Q=0"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/b.json 2> $O/b.err || { echo "BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('0.12 $e', round(d['value']))"
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants > $O/b.json 2> $O/b.err || { echo "KITTI BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('KITTI $e', round(d['value']))"
done; done
echo DONE

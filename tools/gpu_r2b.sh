# new-path parity tests, then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r2b}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/paths.log 2>&1 || { echo PATHS_FAIL; tail -60 $O/paths.log; exit 1; }
tail -3 $O/paths.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_paths.py > $O/all.log 2>&1 || { echo ALL_FAIL; tail -40 $O/all.log; exit 1; }
tail -3 $O/all.log

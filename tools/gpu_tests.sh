# the -m gpu suite (optionally a -k selection) + smoke.  Usage: gpu_tests.sh <tag> ["-k expr"]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tests}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${2:+-k "$2"} > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -5; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log

# repair windows after speculation misses + slack passes: GPU parity tests, then an env A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_ab_env.sh r2r/ab "VO_REPAIR_WIN=64" "VO_REPAIR_WIN=8" "VO_REPAIR_WIN=4" "VO_REPAIR_WIN=8 VO_SLACK=4" "VO_REPAIR_WIN=4 VO_SLACK=8"

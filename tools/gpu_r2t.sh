# pose windows up to 2 extract batches (bounded by the extracted frames): GPU parity tests, env A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_ab_env.sh r2t/ab "VO_WIN=64" "VO_WIN=128" "VO_WIN=128 VO_SLACK=0" "VO_WIN=128 VO_REPAIR_WIN=8"

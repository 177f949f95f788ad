# pair-column stencil: GPU parity tests, then the bench at 4 / 6 / 8 tiles per segment
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_ab_env.sh r2q/ab "VO_STSEG=4" "VO_STSEG=6" "VO_STSEG=8"

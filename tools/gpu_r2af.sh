# select emission via per-word prefixes: GPU parity tests, select stamps, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2af; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 300 python tools/stamps_select.py
bash tools/gpu_ab_env.sh r2af/ab "VO_X=0"

# two extract queues (batch j on queue j % 2, own scratch): parity tests on the eq2 build, env A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2ad; mkdir -p $O
export TMPDIR=/tmp
VO_EXTQ=2 VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_eq2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
export VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_eq2.so
bash tools/gpu_ab_env.sh r2ad/ab "VO_EXTQ=1" "VO_EXTQ=2"

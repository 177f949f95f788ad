# the -m gpu suite against another library build (VO_LIB_PATH), no -x: every failing test listed
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-libtest}; mkdir -p $O
VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$2 timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
grep -E "FAILED|passed|failed" $O/pytest.log | tail -40
echo DONE

# select + describe on a second queue so the next batch's stencil overlaps them: VO_SPLIT=1 (a fifth
# stream) and VO_SPLIT=2 (the trajectory queue) against the default, KITTI and 0.12 m/frame
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w6}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread -k "VO_SPLIT" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab_env.sh ${1:-r5w6}_k "VO_X=0" "VO_SPLIT=1" "VO_SPLIT=2"
bash tools/gpu_ab_env.sh ${1:-r5w6}_012 "VO_X=0" "VO_SPLIT=2" -- --motion 0.12 --sequences 1
echo DONE

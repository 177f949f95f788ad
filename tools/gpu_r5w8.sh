# VO_SPLIT=2 (select + describe on the trajectory queue) with the later RANSAC chunks back on the
# fit queue (VO_RANSAC_Q=0) and with the banded select (VO_SEL1=0): KITTI and 0.12 m/frame
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w8}; mkdir -p $O
bash tools/gpu_ab_env.sh ${1:-r5w8}_k "VO_X=0" "VO_SPLIT=2" "VO_SPLIT=2 VO_RANSAC_Q=0" "VO_SPLIT=2 VO_SEL1=0"
bash tools/gpu_ab_env.sh ${1:-r5w8}_012 "VO_X=0" "VO_SPLIT=2 VO_RANSAC_Q=0" "VO_SPLIT=2 VO_SEL1=0" -- --motion 0.12 --sequences 1
echo DONE

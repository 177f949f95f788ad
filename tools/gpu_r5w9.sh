# the fused RANSAC's one-hypothesis waves (per-frame call / stage API): phase stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w9}; mkdir -p $O
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so STAGE=1 timeout -k 10 200 python3 tools/stamps_ransac.py > $O/stamps_ransac_w1.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_ransac_w1.txt; exit 1; }
cat $O/stamps_ransac_w1.txt
VO_RANSAC_WAVE_HYP=0 VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so STAGE=1 timeout -k 10 200 python3 tools/stamps_ransac.py > $O/stamps_ransac_g8.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_ransac_g8.txt; exit 1; }
cat $O/stamps_ransac_g8.txt
echo DONE

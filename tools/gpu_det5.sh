# MFMA verify build: key and hand-off counters next to the determinism stress
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-det5}; mkdir -p $O
VO_LIB_PATH=$PWD/acs_visual_odometry_amd/libvo_mi355x_mmv.so DET_DBG=1 timeout -k 10 300 python -u tools/det_stress.py 250 0 > $O/det.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det.txt; exit 1; }
grep -E "DIFFERS|seq|frame|full path" $O/det.txt | head -40
grep -vE "wrong 0 of [0-9]+, stale match_j 0 of" $O/det.txt | grep "rep " | head -20
grep "rep 1 " $O/det.txt
echo DONE

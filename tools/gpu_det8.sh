# verify build: select histogram / MFMA / hand-off counters per repeat, ring slots compared
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-det8}; mkdir -p $O
VO_LIB_PATH=$PWD/acs_visual_odometry_amd/libvo_mi355x_mmv.so DET_DBG=1 DET_RING=1 timeout -k 10 500 python -u tools/det_stress.py ${2:-120} 0 > $O/det.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det.txt; exit 1; }
grep -E "full path" $O/det.txt
grep -A3 -E "ring frames differing: [1-9]" $O/det.txt | grep -E "select frame|ring frame " | cut -c1-300 | head -30
grep "rep 1 " $O/det.txt | cut -c1-400
echo DONE

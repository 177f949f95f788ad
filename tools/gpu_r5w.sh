# k_select anatomy in the batched path: pipelined and alone (VO_SERIAL=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w}; mkdir -p $O
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 200 python3 tools/stamps_select_batched.py > $O/sel.txt 2>&1 || { echo STAMPS_FAIL; tail $O/sel.txt; exit 1; }
cat $O/sel.txt
VO_SERIAL=1 VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 200 python3 tools/stamps_select_batched.py > $O/sel_serial.txt 2>&1 || { echo STAMPS_FAIL; tail $O/sel_serial.txt; exit 1; }
cat $O/sel_serial.txt
echo DONE

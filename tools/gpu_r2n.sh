set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2n; mkdir -p $O
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 120 python -u tools/stamps_finalize.py > $O/stamps_fin.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_fin.txt; exit 1; }
cat $O/stamps_fin.txt

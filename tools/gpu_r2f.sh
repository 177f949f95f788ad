set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2f; mkdir -p $O
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 120 python -u tools/stamps_ransac.py > $O/stamps_ransac.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_ransac.txt; exit 1; }
tail -12 $O/stamps_ransac.txt
timeout -k 10 300 python -u -m pytest tests/test_ref_kernels.py -m gpu -x -q -s --timeout 300 --timeout-method thread -k a6 > $O/a6.log 2>&1 || { echo A6_FAIL; tail -30 $O/a6.log; exit 1; }
grep "A.6" $O/a6.log

# per-frame call at the final round-5 build: latency A/B-free rerun, kernel timeline, stage stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5pf_final}; mkdir -p $O
for rep in 1 2; do
  PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  tail -1 $O/pf.txt
done
VO_PF_PROFILE=1 PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pfprof.txt 2>&1 || { echo PFPROF_FAIL; tail $O/pfprof.txt; exit 1; }
tail -3 $O/pfprof.txt
PF_PINNED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o pf -- python3 tools/pf_loop.py 30 > $O/tr.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/tr.txt; exit 1; }
python3 tools/pf_timeline.py $O/tr > $O/pf_timeline.txt 2>&1; cat $O/pf_timeline.txt
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 200 python3 tools/stamps_select_pf.py > $O/stamps_select_pf.txt 2>&1 || { echo STAMPS_FAIL; exit 1; }
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so PF=1 timeout -k 10 200 python3 tools/stamps_describe.py > $O/stamps_describe_pf.txt 2>&1 || { echo STAMPS_FAIL; exit 1; }
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so STAGE=1 timeout -k 10 200 python3 tools/stamps_ransac.py > $O/stamps_ransac_w1.txt 2>&1 || { echo STAMPS_FAIL; exit 1; }
cat $O/stamps_select_pf.txt $O/stamps_describe_pf.txt $O/stamps_ransac_w1.txt
echo DONE

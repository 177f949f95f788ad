# the one-hypothesis wave's Gauss-Jordan pivot by v_readlane (RS_WU_READLANE, default) against the
# LDS pivot row: parity, RANSAC stamps, per-call A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w10}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py tests/test_gpu_reference_sampler.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so STAGE=1 timeout -k 10 200 python3 tools/stamps_ransac.py > $O/stamps_ransac_w1.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_ransac_w1.txt; exit 1; }
cat $O/stamps_ransac_w1.txt
for rep in 1 2; do for lib in libvo_mi355x.so libvo_mi355x_wulds.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$lib $(tail -1 $O/pf.txt)"
done; done
PF_PINNED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o pf -- python3 tools/pf_loop.py 30 > $O/tr.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/tr.txt; exit 1; }
python3 tools/pf_timeline.py $O/tr > $O/pf_timeline.txt 2>&1; cat $O/pf_timeline.txt
echo DONE

# per-frame stencil over PCIe: one 2-byte source load per lane (ST_LD16 build) and the pinned frame
# memory's coherence (VO_HOST_NC) -- parity of the ld16 build, then per-call latency and the
# stencil's duration per (build, allocation) pair, then the batched bench A/B of the two builds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w2}; mkdir -p $O
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_ld16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 200 python3 tools/stamps_select_pf.py > $O/stamps_select_pf.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_select_pf.txt; exit 1; }
cat $O/stamps_select_pf.txt
VO_PF_PROFILE=1 PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pfprof.txt 2>&1 || { echo PFPROF_FAIL; tail $O/pfprof.txt; exit 1; }
tail -3 $O/pfprof.txt
for nc in 0 1 2; do for lib in libvo_mi355x.so libvo_mi355x_ld16.so; do
  VO_HOST_NC=$nc VO_LIB_PATH=acs_visual_odometry_amd/$lib PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "NC=$nc $lib $(tail -1 $O/pf.txt)"
  rm -rf $O/tr
  VO_HOST_NC=$nc VO_LIB_PATH=acs_visual_odometry_amd/$lib PF_PINNED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o pf -- python3 tools/pf_loop.py 30 > $O/tr.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/tr.txt; exit 1; }
  python3 tools/pf_timeline.py $O/tr > $O/tl_${nc}_$lib.txt 2>&1
  grep -E "device span|k_stencil" $O/tl_${nc}_$lib.txt
done; done
bash tools/gpu_ab_libs.sh ${1:-r5w2}_ab "libvo_mi355x.so libvo_mi355x_ld16.so"
echo DONE

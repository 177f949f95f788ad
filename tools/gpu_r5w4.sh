# the per-frame stencil's source rows by two 64-byte loads + ds_bpermute (ST_PF_BPERM build) against
# two overlapping 128-byte loads: parity of the variant, per-call A/B, the stencil's duration
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w4}; mkdir -p $O
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_bp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "per_frame or process_frame or parity or stage" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for lib in libvo_mi355x.so libvo_mi355x_bp.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$lib $(tail -1 $O/pf.txt)"
done; done
for lib in libvo_mi355x.so libvo_mi355x_bp.so; do
  rm -rf $O/tr
  VO_LIB_PATH=acs_visual_odometry_amd/$lib PF_PINNED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o pf -- python3 tools/pf_loop.py 30 > $O/tr.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/tr.txt; exit 1; }
  python3 tools/pf_timeline.py $O/tr > $O/tl_$lib.txt 2>&1
  echo $lib; grep -E "device span|k_stencil" $O/tl_$lib.txt
done
echo DONE

# select bands per frame (VO_SEL_BANDS 8 / 12 / 24 builds): parity of the per-frame paths, per-call
# A/B, and the batched bench (the banded select serves small batches and the stage API too)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w5}; mkdir -p $O
for lib in libvo_mi355x_sb12.so libvo_mi355x_sb24.so; do
VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_parity.py tests/test_select_consistency.py -m gpu -x -q --timeout 300 --timeout-method thread -k "per_frame or process_frame or parity or stage or select" > $O/pytest_$lib.log 2>&1 || { echo PYTEST_FAIL $lib; tail -40 $O/pytest_$lib.log; exit 1; }
echo "$lib $(tail -1 $O/pytest_$lib.log)"
done
for rep in 1 2; do for lib in libvo_mi355x.so libvo_mi355x_sb12.so libvo_mi355x_sb24.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$lib $(tail -1 $O/pf.txt)"
done; done
bash tools/gpu_ab_libs.sh ${1:-r5w5}_ab "libvo_mi355x.so libvo_mi355x_sb12.so"
echo DONE

# the banded / fused select's first key block requested before the boundary-bin scan
# (SEL_KEY_PREFETCH, default) against the loads after it: parity, stamps, per-call and bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w12}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_parity.py tests/test_select_consistency.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 200 python3 tools/stamps_select_pf.py > $O/stamps_select_pf.txt 2>&1 || { echo STAMPS_FAIL; tail $O/stamps_select_pf.txt; exit 1; }
cat $O/stamps_select_pf.txt
for rep in 1 2; do for lib in libvo_mi355x.so libvo_mi355x_nopf.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$lib $(tail -1 $O/pf.txt)"
done; done
bash tools/gpu_ab_libs.sh ${1:-r5w12}_ab "libvo_mi355x.so libvo_mi355x_nopf.so" --width 1920 --height 1080 --max-kpts 4096 --sequences 2 --frames 64
echo DONE

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6h; mkdir -p $O
for rep in 1 2; do for lib in libvo_mi355x_spin.so libvo_mi355x.so; do
  echo "== $lib"; PF_PINNED=1 VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 120 python3 tools/pf_loop.py 60 || exit 1
done; done
VO_REPORT_DIR=$O timeout -k 10 600 python -u -m pytest tests/test_ref_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cat $O/a6_agreement.jsonl
bash tools/gpu_ab_libs.sh r6h_abk "libvo_mi355x_nodw.so libvo_mi355x.so"

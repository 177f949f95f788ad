# the mixed-density select case (fused select: fallback bands and LDS-staged bands in one frame)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w13}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "extract_sizes" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
grep -E "mixed|passed|failed" $O/pytest.log | tail -6
echo DONE

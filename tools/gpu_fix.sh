set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-fix}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_regimes.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_det.sh ${1:-fix}/det VO_MATCH_MFMA=1 VO_MATCH_MFMA=0 VO_MATCH_MFMA=1

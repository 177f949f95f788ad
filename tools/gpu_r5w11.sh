# equal batches per chunk (VO_EVEN=1): parity, then the 0.12 m/frame sequence and KITTI A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w11}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread -k "VO_EVEN" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab_env.sh ${1:-r5w11}_012 "VO_X=0" "VO_EVEN=1" -- --motion 0.12 --sequences 1
bash tools/gpu_ab_env.sh ${1:-r5w11}_005 "VO_X=0" "VO_EVEN=1" -- --motion 0.05 --sequences 1
bash tools/gpu_ab_env.sh ${1:-r5w11}_k "VO_X=0" "VO_EVEN=1"
echo DONE

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/bisect; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -v --timeout 120 --timeout-method thread -k "config4_full_path_1080p" > $O/a.log 2>&1; rc=$?; tail -5 $O/a.log; echo "rc=$rc"

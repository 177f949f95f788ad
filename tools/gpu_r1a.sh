set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r1a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r1a/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r1a/pytest.log; exit 1; }
tail -3 gpurun_out/r1a/pytest.log
timeout -k 10 300 python -u bench.py --breakdown > gpurun_out/r1a/bench.json 2> gpurun_out/r1a/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r1a/bench.err; exit 1; }
cat gpurun_out/r1a/bench.json
cat gpurun_out/r1a/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1a/prof -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/r1a/prof_bench.json 2>&1 || { echo PROF_FAIL; exit 1; }
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 120 python tools/stamps.py > gpurun_out/r1a/stamps.txt 2>&1 || echo STAMPS_FAIL
cat gpurun_out/r1a/stamps.txt

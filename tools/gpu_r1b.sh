set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r1b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu --breakdown > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json; cat $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o trace -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/prof_bench.json 2>&1 || { echo PROF_FAIL; exit 1; }
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so timeout -k 10 120 python tools/stamps_frame.py > $O/stamps_frame.txt 2>&1 || echo STAMPS_FAIL
cat $O/stamps_frame.txt

# round evidence: all -m gpu tests, smoke, default bench (CPU leg), 1080p bench, and the
# rocprofv3 duration + FETCH_SIZE / WRITE_SIZE profiles of both configs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-round}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python -u bench.py --breakdown > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json; cat $O/bench.err
timeout -k 10 300 python -u bench.py --no-cpu --width 1920 --height 1080 --max-kpts 4096 --breakdown > $O/bench_1080.json 2> $O/bench_1080.err || { echo BENCH1080_FAIL; tail -20 $O/bench_1080.err; exit 1; }
cat $O/bench_1080.json; cat $O/bench_1080.err
bash tools/profile.sh $O/prof_kitti > $O/prof_kitti.log 2>&1 || { echo PROF_FAIL; tail $O/prof_kitti.log; exit 1; }
bash tools/profile.sh $O/prof_1080 --width 1920 --height 1080 --max-kpts 4096 > $O/prof_1080.log 2>&1 || { echo PROF1080_FAIL; tail $O/prof_1080.log; exit 1; }
echo DONE

# round evidence: all -m gpu tests, smoke, the default bench (CPU leg + variants), the rocprofv3
# duration + FETCH_SIZE / WRITE_SIZE / VALU profiles of the three bench configs, the FETCH_SIZE
# calibration.  Usage: gpu_round.sh <tag> [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-round}; mkdir -p $O
if [ -z "$2" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
fi
timeout -k 10 600 python -u bench.py --breakdown > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('VALUE',round(d['value']),'dominant',d['roofline']['kernel']);print(json.dumps(d['variants'],indent=0)[:3000]);print(json.dumps(d['cpu_baseline']))"
bash tools/profile.sh $O/prof_kitti > $O/prof_kitti.log 2>&1 || { echo PROF_FAIL; tail $O/prof_kitti.log; exit 1; }
bash tools/profile.sh $O/prof_1080 --width 1920 --height 1080 --max-kpts 4096 --frames 64 > $O/prof_1080.log 2>&1 || { echo PROF1080_FAIL; tail $O/prof_1080.log; exit 1; }
bash tools/profile.sh $O/prof_1080_512 --width 1920 --height 1080 --max-kpts 4096 --frames 64 --match-bits 512 > $O/prof_1080_512.log 2>&1 || { echo PROF512_FAIL; tail $O/prof_1080_512.log; exit 1; }
echo DONE

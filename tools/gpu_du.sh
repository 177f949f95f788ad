# describe variants: parity, the determinism stress, alternating KITTI lines (args: out-tag other-lib)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-du}; mkdir -p $O
OTHER=$2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_regimes.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/det_stress.py 12 6 > $O/det.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det.txt; exit 1; }
grep -E "differ|DIFFERS|seq|frame" $O/det.txt | head -40
for rep in 1 2 3; do
for lib in libvo_mi355x.so $OTHER; do
  VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants --steps 10 > $O/b.json 2> $O/b.err || { echo FAIL "$lib"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('kitti', '$lib', round(d['value']), d['determinism']['timed_rows_equal_warmup_rows'], d['determinism']['gathered_rows_equal_separate_runs'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
echo DONE

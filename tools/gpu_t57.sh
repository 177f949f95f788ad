# stencil tile geometry: parity with the default build, then alternating KITTI and 1080p lines
# against a second library build (args: out-tag other-lib)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-t57}; mkdir -p $O
OTHER=$2
timeout -k 10 840 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_parity.py tests/test_gpu_regimes.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
for lib in libvo_mi355x.so $OTHER; do
  VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants --steps 10 > $O/b.json 2> $O/b.err || { echo FAIL "$lib"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('kitti', '$lib', round(d['value']), d['determinism']['timed_rows_equal_warmup_rows'], d['determinism']['gathered_rows_equal_separate_runs'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
for rep in 1 2; do
for lib in libvo_mi355x.so $OTHER; do
  VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants --steps 5 --width 1920 --height 1080 --max-kpts 4096 --frames 64 --sequences 2 --match-bits 32 > $O/b.json 2> $O/b.err || { echo FAIL "$lib"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('1080', '$lib', round(d['value']), d['determinism']['timed_rows_equal_warmup_rows'], d['determinism']['gathered_rows_equal_separate_runs'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
echo DONE

# banded select: extract parity (every size, periodic boundary bins) + trajectory tests, then A/B
# of VO_SEL1 (single-workgroup select) at KITTI and 1920x1080
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-sel}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for e in VO_SEL1=1 VO_SEL1=0; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --no-check --steps 10 > $O/b.json 2> $O/b.err || { echo FAIL "$e"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('kitti', '$e', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --no-check --steps 5 --width 1920 --height 1080 --max-kpts 4096 --frames 64 > $O/b.json 2> $O/b.err || { echo FAIL "$e"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('1080', '$e', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
echo DONE

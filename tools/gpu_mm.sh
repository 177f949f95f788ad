# MFMA matcher: operand-map probe, parity (every -m gpu test of the parity / golden / paths files),
# then alternating bench lines with the VALU matcher (VO_MATCH_MFMA=0) and the MFMA one
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-mm}; mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k mfma --timeout 60 > $O/mfma.log 2>&1; tail -3 $O/mfma.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_regimes.py tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for e in VO_MATCH_MFMA=0 VO_MATCH_MFMA=1; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --no-check --steps 10 > $O/b.json 2> $O/b.err || { echo FAIL "$e"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('kitti', '$e', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --no-check --steps 5 --motion 0.12 --sequences 1 > $O/b.json 2> $O/b.err || { echo FAIL "$e"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('0.12', '$e', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
timeout -k 10 200 python3 tools/pf_loop.py 60
echo DONE

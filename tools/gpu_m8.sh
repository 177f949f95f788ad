# matchers with prefetched chunks: parity, then KITTI and 1920x1080 lines, VALU vs MFMA matchers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-m8}; mkdir -p $O
timeout -k 10 840 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_parity.py tests/test_gpu_regimes.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for e in VO_MATCH_MFMA=0 VO_MATCH_MFMA=1; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --steps 10 > $O/b.json 2> $O/b.err || { echo FAIL "$e"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('kitti', '$e', round(d['value']), d['determinism']['timed_rows_equal_warmup_rows'], d['determinism']['gathered_rows_equal_separate_runs'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
for bits in 512 32; do
for e in VO_MATCH_MFMA=0 VO_MATCH_MFMA=1; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --steps 5 --width 1920 --height 1080 --max-kpts 4096 --frames 64 --sequences 2 --match-bits $bits > $O/b.json 2> $O/b.err || { echo FAIL "$e"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('1080', $bits, '$e', round(d['value']), d['determinism']['timed_rows_equal_warmup_rows'], d['determinism']['gathered_rows_equal_separate_runs'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
timeout -k 10 200 python3 tools/pf_loop.py 60
echo DONE

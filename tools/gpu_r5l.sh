# small batches through the banded select: parity of the batched paths, 0.12 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5l}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_regimes.py tests/test_gpu_paths.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for e in "VO_SEL_SMALL=16" "VO_SEL_SMALL=0" "VO_SEL_LDS_KB=64"; do
  env $e timeout -k 10 200 python -u bench.py --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/b.json 2> $O/b.err || { echo "BENCH_FAIL"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('0.12 $e', round(d['value']), {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-variants --motion 0.12 --sequences 1 > $O/trace.json 2>&1 || { echo TRACE_FAIL; exit 1; }
echo DONE

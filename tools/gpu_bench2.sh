# default and 1920x1080/N=4096 bench lines (no CPU leg), plus the pipeline-sensitive parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-b2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "trajectory or pipelined or batched or skip" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu --steps 40 > $O/k.json 2> $O/k.err || { echo BENCH_FAIL; tail -5 $O/k.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --steps 20 --width 1920 --height 1080 --max-kpts 4096 > $O/x.json 2> $O/x.err || { echo BENCHX_FAIL; tail -5 $O/x.err; exit 1; }
python3 -c "import json;[print(n, round(json.load(open('$O/'+n+'.json'))['value'],1)) for n in ('k','x')]"

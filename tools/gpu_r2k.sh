set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread -k "windowed or host or sequence or leak or event or trajectory or batched or skip or config" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu --no-variants > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail $O/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));print(round(d['value']), d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-variants > $O/tr.json 2>&1 || { echo TRACE_FAIL; tail $O/tr.json; exit 1; }

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread -k "leak or event or sequence" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab_env.sh r2l_ev "VO_EVENT_WAIT=0" "VO_EVENT_WAIT=1" || exit 1
VO_EVENT_WAIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-variants > $O/tr.json 2>&1 || { echo TRACE_FAIL; tail $O/tr.json; exit 1; }
python3 tools/pass_timeline.py $O/tr/trace_kernel_trace.csv | head -30

# per-frame parity (knobs + leak sequence + smoke) and the per-frame call's latency / trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_reference_sampler.py tests/test_gpu_paths.py tests/test_gpu_matchers.py tests/test_gpu_parity.py tests/test_facade.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_PF_PROFILE=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
PF_PINNED=1 VO_PF_PROFILE=1 timeout -k 10 200 python3 tools/pf_loop.py 60 >> $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
cat $O/pf.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/pftrace -o pf -- python3 tools/pf_loop.py 30 > $O/pftrace.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/pftrace.txt; exit 1; }
python3 tools/pf_timeline.py $O/pftrace > $O/pf_timeline.txt 2>&1; cat $O/pf_timeline.txt
echo DONE

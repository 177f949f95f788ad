# latency RANSAC: later chunk on <= 60 workgroups; one vs eight hypotheses per wave (A/B); parity
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5r}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_sampler.py tests/test_gpu_paths.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for e in "VO_RANSAC_WAVE_HYP=1" "VO_RANSAC_WAVE_HYP=0" "VO_RANSAC_WAVE_HYP=1 VO_RANSAC_WG1=1000"; do
  env $e PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$e $(tail -1 $O/pf.txt)"
done; done
PF_PINNED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pftrace -o pf -- python3 tools/pf_loop.py 30 > $O/pftrace.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/pftrace.txt; exit 1; }
python3 tools/pf_timeline.py $O/pftrace > $O/pf_timeline.txt 2>&1; cat $O/pf_timeline.txt
echo DONE

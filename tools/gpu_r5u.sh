# per-frame call: poll the pinned row's done marker instead of the stream wait (A/B); parity of the
# per-frame paths
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5u}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_parity.py tests/test_gpu_reference_sampler.py tests/test_gpu_matchers.py tests/test_facade.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do for e in "VO_PF_POLL=1" "VO_PF_POLL=0"; do
  env $e PF_PINNED=1 VO_PF_PROFILE=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$e $(grep 'rep 1' $O/pf.txt) $(grep 'host phases' $O/pf.txt)"
  env $e timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$e $(tail -1 $O/pf.txt)"
done; done
echo DONE

# per-frame stencil segments 1 / 2 / 4 tile rows (A/B) with parity of the knob
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5y}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q -k "per_frame_knobs" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_PF_SEGT=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py -m gpu -x -q -k "per_frame_call_from_pinned" --timeout 200 --timeout-method thread > $O/pytest4.log 2>&1 || { echo PYTEST4_FAIL; tail -40 $O/pytest4.log; exit 1; }
tail -1 $O/pytest4.log
for rep in 1 2; do for e in "VO_PF_SEGT=1" "VO_PF_SEGT=4"; do
  env $e PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$e $(tail -1 $O/pf.txt)"
done; done
VO_PF_SEGT=4 PF_PINNED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pftrace -o pf -- python3 tools/pf_loop.py 30 > $O/pftrace.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/pftrace.txt; exit 1; }
python3 tools/pf_timeline.py $O/pftrace > $O/pf_timeline.txt 2>&1; head -4 $O/pf_timeline.txt
echo DONE

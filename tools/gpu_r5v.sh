# describe_pf term waves generated at compile time: parity, stamps, per-frame A/B against the table form
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5v}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_parity.py tests/test_facade.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VO_LIB_PATH=acs_visual_odometry_amd/libvo_mi355x_stamps.so PF=1 timeout -k 10 200 python3 tools/stamps_describe.py > $O/stamps_describe_pf.txt 2>&1 || { echo STAMPS_DS_FAIL; tail $O/stamps_describe_pf.txt; exit 1; }
cat $O/stamps_describe_pf.txt
for rep in 1 2; do for lib in libvo_mi355x.so libvo_mi355x_dpold.so; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib PF_PINNED=1 timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
  echo "$lib $(tail -1 $O/pf.txt)"
done; done
PF_PINNED=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pftrace -o pf -- python3 tools/pf_loop.py 30 > $O/pftrace.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/pftrace.txt; exit 1; }
python3 tools/pf_timeline.py $O/pftrace > $O/pf_timeline.txt 2>&1; cat $O/pf_timeline.txt
echo DONE

# per-frame call path (vo_process_frame): per-call latency, then a kernel + copy trace of it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pf}; mkdir -p $O
timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
cat $O/pf.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/pftrace -o pf -- python3 tools/pf_loop.py 30 > $O/pftrace.txt 2>&1 || { echo PFTRACE_FAIL; tail $O/pftrace.txt; exit 1; }
python3 tools/pf_timeline.py $O/pftrace > $O/pf_timeline.txt 2>&1; cat $O/pf_timeline.txt
echo DONE

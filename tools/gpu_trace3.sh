# kernel traces: the headline bench (queue timeline) and the per-frame call path
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tr3}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-variants --no-check > $O/trace.json 2>&1 || { echo TRACE_FAIL; tail $O/trace.json; exit 1; }
python3 tools/step_timeline.py $O/trace/tr_kernel_trace.csv > $O/steps.txt 2>&1 || true
timeout -k 10 200 python3 tools/pf_loop.py 60 > $O/pf.txt 2>&1 || { echo PF_FAIL; tail $O/pf.txt; exit 1; }
cat $O/pf.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/pftrace -o pf -- python3 tools/pf_loop.py 30 > $O/pftrace.txt 2>&1 || { echo PFTRACE_FAIL; exit 1; }
echo DONE

# kernel trace of the headline bench (queue busy fractions, pass anatomy)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tr4}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr -- python3 bench.py --steps 4 --warmup 2 --no-cpu --no-variants --no-check > $O/trace.json 2>&1 || { echo TRACE_FAIL; tail $O/trace.json; exit 1; }
python3 tools/step_timeline.py $O/trace/tr_kernel_trace.csv > $O/steps.txt 2>&1 || true
head -60 $O/steps.txt
echo DONE

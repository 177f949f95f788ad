set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r2j; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-variants > $O/tr.json 2>&1 || { echo TRACE_FAIL; tail $O/tr.json; exit 1; }
python3 tools/pass_timeline.py $O/tr/trace_kernel_trace.csv
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr12 -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-variants --motion 0.12 --sequences 2 > $O/tr12.json 2>&1 || { echo TRACE_FAIL; tail $O/tr12.json; exit 1; }
python3 tools/pass_timeline.py $O/tr12/trace_kernel_trace.csv

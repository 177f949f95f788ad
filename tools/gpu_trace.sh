# kernel trace of the headline bench (8 sequences) for the queue timeline:
#   gpu_trace.sh <tag> [bench args]   then tools/step_timeline.py gpurun_out/<tag>/trace/tr_kernel_trace.csv
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu --no-variants "$@" > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('VALUE',round(d['value']))"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-variants "$@" > $O/trace.json 2>&1 || { echo TRACE_FAIL; exit 1; }
echo TRACE_OK

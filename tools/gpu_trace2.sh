# kernel trace of the headline bench (no check runs) for the per-queue busy / gap analysis (tools/steps.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tr}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-variants --no-check > $O/prof_bench.json 2>&1 || { echo PROF_FAIL; tail $O/prof_bench.json; exit 1; }
echo OK

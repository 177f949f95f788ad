# trace of short bench runs at a few batch sizes + per-step phase breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-steps}; mkdir -p $O
for b in 64; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p$b -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --batch $b > $O/b$b.json 2>&1 || { echo PROF_FAIL; exit 1; }
echo "batch $b"; python3 tools/steps.py $O/p$b/trace_kernel_trace.csv
done

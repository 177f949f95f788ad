# rocprofv3 duration + PMC profiles of the default workload and of the 1920x1080/4096 stress
# config, plus their bench lines (tools/profile.sh per workload)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r1c}
bash tools/profile.sh gpurun_out/prof_$T || { echo PROF_FAIL; exit 1; }
bash tools/profile.sh gpurun_out/prof_${T}x --width 1920 --height 1080 --max-kpts 4096 || { echo PROFX_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --width 1920 --height 1080 --max-kpts 4096 --breakdown > gpurun_out/prof_${T}x/bench.json 2> gpurun_out/prof_${T}x/bench.err || { echo BENCHX_FAIL; exit 1; }
cat gpurun_out/prof_${T}x/bench.json
python3 tools/timeline.py gpurun_out/prof_$T/stats_kernel_trace.csv | head -14

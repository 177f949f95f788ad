# Determinism evidence on the GPU box (replaces round 3's one-off gpu_det*/gpu_m*/gpu_trace* scripts).
#   tools/gpu_det.sh <tag> <repeats> "<lib>[:ENV=V,...] ..."
# For each library (acs_visual_odometry_amd/<lib>) and environment: tools/det_stress.py <repeats>
# (the bench's 8 x 200-frame stream repeated under changing kernel-timing modes, ring slots
# compared), with the device buffer layout printed first.  Logs: gpurun_out/<tag>/det_<n>.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-det}; REPS=${2:-100}; RUNS=${3:-"libvo_mi355x.so:VO_MATCH_MFMA=1"}; XREPS=${4:-0}
O=gpurun_out/$TAG; mkdir -p $O
if [ -x acs_visual_odometry_amd/bin/buffer_range_probe ]; then
  timeout -k 10 60 acs_visual_odometry_amd/bin/buffer_range_probe > $O/buffer_range_probe.txt || { echo PROBE_FAIL; exit 1; }
  cat $O/buffer_range_probe.txt
fi
n=0
for run in $RUNS; do
  lib=${run%%:*}; envs=""; [ "$run" != "$lib" ] && envs=$(echo ${run#*:} | tr ',' ' ')
  n=$((n + 1))
  echo "== $lib $envs ($REPS repeats)"
  env $envs VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib DET_RING=1 timeout -k 10 600 python -u tools/det_stress.py $REPS $XREPS > $O/det_$n.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det_$n.txt; exit 1; }
  grep -E "full path|extract:|^diag:" $O/det_$n.txt
done
echo DONE

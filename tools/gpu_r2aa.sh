# timeline trace of the current build + stencil segment / window A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_trace.sh r2aa || exit 1
bash tools/gpu_ab_env.sh r2aa/ab "VO_STSEG=4" "VO_STSEG=6" "VO_STSEG=2"

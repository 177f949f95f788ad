set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r5f.sh r5f && bash tools/gpu_r5g.sh r5g

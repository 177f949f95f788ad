# hardware queues: select + describe on a fifth stream with 8 hardware queues per process
# (GPU_MAX_HW_QUEUES=8 VO_SPLIT=1), two extract queues, and the frame batch 64 / 96 / 128
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5w7}; mkdir -p $O
bash tools/gpu_ab_env.sh ${1:-r5w7}_k "VO_X=0" "GPU_MAX_HW_QUEUES=8 VO_SPLIT=1" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=8 VO_EXTQ=2"
bash tools/gpu_ab_env.sh ${1:-r5w7}_012 "VO_X=0" "GPU_MAX_HW_QUEUES=8 VO_SPLIT=1" -- --motion 0.12 --sequences 1
bash tools/gpu_ab_args.sh ${1:-r5w7}_b "--batch 64" "--batch 96" "--batch 128"
echo DONE

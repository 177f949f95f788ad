set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_ab_libs.sh abm "libvo_mi355x.so libvo_mi355x_oldm.so" --sequences 4 || exit 1
VO_SERIAL=1 bash tools/gpu_ab_libs.sh abms "libvo_mi355x.so libvo_mi355x_oldm.so" --sequences 2 || exit 1
bash tools/gpu_ab_libs.sh abmx "libvo_mi355x.so libvo_mi355x_oldm.so" --width 1920 --height 1080 --max-kpts 4096 --frames 64 --sequences 4 || exit 1

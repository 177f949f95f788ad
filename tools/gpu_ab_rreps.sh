# RANSAC later-chunk reps A/B + parity: gpu_ab_rreps.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 4 8; do
  VO_RREPS=$r timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ransac or trajectory or windowed" > gpurun_out/t_r$r.log 2>&1 || { echo FAIL $r; tail -20 gpurun_out/t_r$r.log; exit 1; }
  echo "reps $r: $(tail -1 gpurun_out/t_r$r.log)"
done
bash tools/gpu_ab_env.sh ab_rreps "VO_RREPS=1" "VO_RREPS=4" --steps 10 && bash tools/gpu_ab_env.sh ab_rreps8 "VO_RREPS=8" "VO_RREPS=4" --steps 10

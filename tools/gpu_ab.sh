# repeat the pipeline-sensitive GPU parity tests against one or more library builds (AB_LIBS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
for lib in ${AB_LIBS:-libvo_mi355x.so libvo_mi355x.so libvo_mi355x.so}; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "trajectory or pipelined or batched or skip" > $O/$lib.log 2>&1; echo "$lib rc=$? $(tail -1 $O/$lib.log)"
done

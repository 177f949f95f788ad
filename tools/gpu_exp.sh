# A/B timing of experiment builds (bench --no-cpu, per-kernel breakdown)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-exp}; mkdir -p $O; shift
for lib in libvo_mi355x.so "$@"; do
  VO_LIB_PATH=acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --breakdown > $O/b.json 2> $O/b.err || { echo FAIL $lib; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('$lib', round(d['value'],1), {k: round(v*1e3,2) for k,v in d['kernels_ms_per_frame'].items()})"
done

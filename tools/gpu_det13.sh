# which stencil/select instructions the run-to-run differences need: verify-build amplifier on the
# ablations, then the default-build candidates (stress + bench line)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-det13}; mkdir -p $O
for lib in libvo_mi355x_mmve.so libvo_mi355x_mmvd.so; do
  echo "== amplifier $lib"
  VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib DET_DBG=1 DET_RING=1 timeout -k 10 300 python -u tools/det_stress.py 40 0 > $O/det_$lib.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det_$lib.txt; exit 1; }
  grep -E "full path" $O/det_$lib.txt
  grep -oE "ring frames differing: [0-9]+" $O/det_$lib.txt | awk '{s+=$4} END {print "ring frames differing, total over repeats:", s}'
done
for lib in libvo_mi355x_nodot.so libvo_mi355x_noasm.so; do
  echo "== default-build candidate $lib"
  VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib DET_RING=1 timeout -k 10 300 python -u tools/det_stress.py 200 0 > $O/det_$lib.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det_$lib.txt; exit 1; }
  grep -E "full path" $O/det_$lib.txt
done
for lib in libvo_mi355x.so libvo_mi355x_nodot.so libvo_mi355x_noasm.so; do
  VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants --steps 10 > $O/b.json 2> $O/b.err || { echo FAIL "$lib"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('kitti', '$lib', round(d['value']), d['determinism']['timed_rows_equal_warmup_rows'], d['determinism']['gathered_rows_equal_separate_runs'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
echo DONE

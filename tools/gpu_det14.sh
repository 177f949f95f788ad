# MFMA results in AGPRs (no -amdgpu-mfma-vgpr-form): verify-build amplifier, default-build stress, bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-det14}; mkdir -p $O
for lib in libvo_mi355x_agprv.so; do
  echo "== amplifier $lib"
  VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib DET_DBG=1 DET_RING=1 timeout -k 10 300 python -u tools/det_stress.py 40 0 > $O/det_$lib.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det_$lib.txt; exit 1; }
  grep -E "full path" $O/det_$lib.txt
  grep -oE "ring frames differing: [0-9]+" $O/det_$lib.txt | awk '{s+=$4} END {print "ring frames differing, total over repeats:", s}'
done
for lib in libvo_mi355x_agpr.so; do
  echo "== default-build candidate $lib"
  VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib DET_RING=1 timeout -k 10 300 python -u tools/det_stress.py 250 0 > $O/det_$lib.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det_$lib.txt; exit 1; }
  grep -E "full path" $O/det_$lib.txt
done
for rep in 1 2; do
for lib in libvo_mi355x.so libvo_mi355x_agpr.so; do
  VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib timeout -k 10 200 python -u bench.py --no-cpu --no-variants --steps 10 > $O/b.json 2> $O/b.err || { echo FAIL "$lib"; tail -5 $O/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b.json'));print('kitti', '$lib', round(d['value']), d['determinism']['timed_rows_equal_warmup_rows'], d['determinism']['gathered_rows_equal_separate_runs'], {k: v['us_per_frame'] for k, v in d['kernels'].items()})"
done
done
echo DONE

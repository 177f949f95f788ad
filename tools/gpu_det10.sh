# verify builds without parts of the stencil's hand-written asm: ring frames differing per repeat
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-det10}; mkdir -p $O
shift
for lib in "$@"; do
  echo "== $lib"
  VO_LIB_PATH=$PWD/acs_visual_odometry_amd/$lib DET_DBG=1 DET_RING=1 timeout -k 10 300 python -u tools/det_stress.py 40 0 > $O/det_$lib.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det_$lib.txt; exit 1; }
  grep -E "full path" $O/det_$lib.txt
  grep -oE "ring frames differing: [0-9]+" $O/det_$lib.txt | awk '{s+=$4} END {print "ring frames differing, total over repeats:", s}'
done
echo DONE

# determinism stress with the extracted ring slots compared after every repeat
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-det6}; mkdir -p $O
DET_RING=1 timeout -k 10 400 python -u tools/det_stress.py ${2:-120} 0 > $O/det.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det.txt; exit 1; }
grep -E "DIFFERS|ring frame|full path" $O/det.txt | head -40
grep -E "ring frames differing: [1-9]" $O/det.txt | head -10
grep "rep 1 " $O/det.txt
echo DONE

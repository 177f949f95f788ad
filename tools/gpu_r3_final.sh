# round-3 final build: full -m gpu suite + smoke, the per-frame call trace, then the determinism stress
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3final}; mkdir -p $O
bash tools/gpu_r3_tests.sh ${1:-r3final} || exit 1
timeout -k 10 300 python -u tools/det_stress.py 250 0 > $O/det.txt 2>&1 || { echo DET_FAIL; tail -20 $O/det.txt; exit 1; }
grep -E "DIFFERS|full path" $O/det.txt | head -12
echo DONE

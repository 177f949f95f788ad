# round evidence from one build: the full -m gpu suite + smoke, then the profiles and the bench
# (tools/gpu_evidence.sh).  Usage: gpu_final.sh <round: r6> <tag> [workloads...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-r6}; T=${2:-${R}final}; shift 2
O=gpurun_out/$T; mkdir -p $O
VO_REPORT_DIR=$O timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
bash tools/gpu_evidence.sh $R ${T}_ev ${@:-kitti kitti_012 1080 1080_512} bench
